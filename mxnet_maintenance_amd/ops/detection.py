"""Detection operators (placeholder module; filled in below)."""
