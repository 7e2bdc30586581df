"""ORACLE — test infrastructure only (see ref_unet.py header)."""
