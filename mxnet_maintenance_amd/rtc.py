"""rtc (being implemented)."""
