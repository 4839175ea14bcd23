"""mivod.ops."""
