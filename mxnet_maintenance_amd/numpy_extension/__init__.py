"""numpy_extension (being implemented)."""
