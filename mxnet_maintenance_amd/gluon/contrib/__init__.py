"""gluon/contrib (being implemented)."""
