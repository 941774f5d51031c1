"""Minimal SimCLR model pieces (projection head + synthetic trainer)."""
