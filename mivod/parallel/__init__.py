"""mivod.parallel."""
