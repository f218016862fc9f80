"""io (being implemented)."""
