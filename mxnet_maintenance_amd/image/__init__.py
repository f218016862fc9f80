"""image (being implemented)."""
