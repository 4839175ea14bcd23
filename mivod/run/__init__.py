"""mivod.run."""
