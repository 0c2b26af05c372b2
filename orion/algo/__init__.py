"""``orion.algo``: plugin base classes for third-party algorithms."""
