"""visualization (being implemented)."""
