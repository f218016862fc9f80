"""model (being implemented)."""
