"""Python runners of the on-device plugins (oracles for the native samplers)."""
