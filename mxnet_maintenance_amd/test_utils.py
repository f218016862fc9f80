"""test_utils (being implemented)."""
