"""mivod.data."""
