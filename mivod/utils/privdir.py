"""Private per-user staging directories (MIOpen find-db, TunableOp tables).

The ranks of one node share the directory, so its name is predictable —
which is only safe if nobody else can own or write it: it is created 0700,
and an existing path that is not a directory owned by this user with no
group/other permissions is never used (a fresh ``mkdtemp`` is used instead).
"""
from __future__ import annotations

import os
import stat
import tempfile


def private_tmp(name: str) -> str:
    d = os.path.join(tempfile.gettempdir(), f"mivod_{name}_{os.getuid()}")
    try:
        os.mkdir(d, 0o700)
    except FileExistsError:
        pass
    except OSError:
        return tempfile.mkdtemp(prefix=f"mivod_{name}_")
    st = os.lstat(d)
    if not stat.S_ISDIR(st.st_mode) or st.st_uid != os.getuid() or (st.st_mode & 0o077):
        return tempfile.mkdtemp(prefix=f"mivod_{name}_")
    return d
