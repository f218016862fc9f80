"""numpy (being implemented)."""
