"""profiler (being implemented)."""
