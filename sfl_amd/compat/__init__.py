"""Adapters for code written against the reference's own packages."""
