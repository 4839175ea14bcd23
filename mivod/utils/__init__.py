"""mivod.utils."""
