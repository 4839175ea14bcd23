"""mivod.keras."""
