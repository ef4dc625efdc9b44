"""Synthetic input generation for tests and bench (not product, not oracle)."""
