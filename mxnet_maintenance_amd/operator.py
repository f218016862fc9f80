"""operator (being implemented)."""
