"""Utilities package."""
