"""Drop-in for the reference managers package (managers/extractor.py)."""
