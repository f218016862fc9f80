"""module (being implemented)."""
