"""monitor (being implemented)."""
