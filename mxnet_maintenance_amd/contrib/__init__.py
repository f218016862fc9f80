"""contrib (being implemented)."""
