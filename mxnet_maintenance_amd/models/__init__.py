"""models (being implemented)."""
