"""mivod.common."""
