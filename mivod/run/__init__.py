"""mivod launcher (``mivodrun`` / ``horovodrun`` compatible)."""
from .launcher import assign_slots, launch, main, parse_hostfile, parse_hosts

__all__ = ["main", "launch", "assign_slots", "parse_hosts", "parse_hostfile"]
