"""callback (being implemented)."""
