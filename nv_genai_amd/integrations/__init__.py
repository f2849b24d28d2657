"""Adapters for third-party frameworks the reference integrates with (integrations/ in the reference)."""
