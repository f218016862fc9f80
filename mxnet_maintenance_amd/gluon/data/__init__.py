"""gluon/data (being implemented)."""
