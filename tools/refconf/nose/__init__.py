"""Minimal stand-in for the parts of ``nose`` the reference unit tests import."""
