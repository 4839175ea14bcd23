"""mivod.models."""
