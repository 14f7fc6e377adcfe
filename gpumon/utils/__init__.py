"""Small shared helpers (statistics, timing)."""
