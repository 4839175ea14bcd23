"""``mivodrun`` / ``horovodrun`` — process launcher.

Replaces the reference's ``mpirun --allow-run-as-root -np N --hostfile H
-bind-to none -map-by slot -x NCCL_DEBUG=INFO -mca pml ob1 -mca btl ^openib
python ...`` (/root/reference/README.md:57, .ps_project/distributed-keras-sample.yaml:8)
without MPI: one process per GPU slot, rank-major over hosts, with the
environment contract every mivod / torch.distributed program reads
(``HOROVOD_{RANK,SIZE,LOCAL_RANK,LOCAL_SIZE,CROSS_RANK,CROSS_SIZE}`` plus
torchrun's ``RANK/WORLD_SIZE/LOCAL_RANK/LOCAL_WORLD_SIZE/MASTER_ADDR/MASTER_PORT``).

* accepts horovodrun flags (``-np``, ``-H host:slots,...``, ``--hostfile``
  with ``host slots=N`` or ``host:N`` lines, tuning flags mapped to
  ``HOROVOD_*`` env) and tolerates mpirun flags (``-bind-to``, ``-map-by``,
  ``-mca k v``, ``--allow-run-as-root``, ``--oversubscribe``, ``-x VAR[=v]``,
  ``--tag-output``), so the reference's command lines work with ``mpirun``
  replaced by ``mivodrun``;
* local slots are spawned directly, remote ones over ``ssh``;
* output is prefixed per rank (``[1,0]<stdout>:`` mpirun style) when
  ``--tag-output`` is given or size > 1;
* if any rank exits non-zero, the others are terminated (mpirun semantics) and
  the launcher exits with that code;
* horovodrun extras: ``--check-build`` (what this install provides),
  ``--config-file`` (horovodrun's YAML: params / autotune / timeline /
  stall_check / logging sections; command-line flags win), ``--output-filename
  DIR`` (per-rank ``DIR/rank.N/{stdout,stderr}`` copies), ``--disable-cache``,
  ``--network-interface IF`` (-> ``NCCL_SOCKET_IFNAME`` / ``GLOO_SOCKET_IFNAME``).
"""
from __future__ import annotations

import argparse
import os
import shlex
import signal
import socket
import subprocess
import sys
import threading
import time
from dataclasses import dataclass
from typing import Dict, List, Optional, Sequence, Tuple

LOCAL_NAMES = {"localhost", "127.0.0.1", "::1"}


@dataclass
class Slot:
    host: str
    rank: int
    local_rank: int
    local_size: int
    cross_rank: int
    cross_size: int


def parse_hosts(spec: str) -> List[Tuple[str, int]]:
    """'a:4,b:2' -> [('a', 4), ('b', 2)]; a bare host counts 1 slot."""
    out = []
    for item in spec.split(","):
        item = item.strip()
        if not item:
            continue
        if ":" in item:
            h, n = item.rsplit(":", 1)
            out.append((h, int(n)))
        else:
            out.append((item, 1))
    return out


def parse_hostfile(path: str) -> List[Tuple[str, int]]:
    """mpirun / horovodrun hostfiles: 'host slots=N', 'host:N' or 'host'."""
    out = []
    with open(path) as f:
        for line in f:
            line = line.split("#", 1)[0].strip()
            if not line:
                continue
            parts = line.split()
            host, slots = parts[0], 1
            if ":" in host:
                host, n = host.rsplit(":", 1)
                slots = int(n)
            for p in parts[1:]:
                if p.startswith("slots="):
                    slots = int(p.split("=", 1)[1])
                elif p.startswith("max_slots=") and slots == 1:
                    pass
            out.append((host, slots))
    return out


def assign_slots(hosts: List[Tuple[str, int]], np: int) -> List[Slot]:
    """Fill hosts slot by slot (``-map-by slot``), rank-major."""
    total = sum(n for _, n in hosts)
    if np > total:
        raise ValueError(f"-np {np} exceeds the {total} available slots ({hosts})")
    placed: List[Tuple[str, int]] = []
    for h, n in hosts:
        for lr in range(n):
            if len(placed) == np:
                break
            placed.append((h, lr))
    used_hosts = []
    for h, _ in placed:
        if h not in used_hosts:
            used_hosts.append(h)
    local_sizes = {h: sum(1 for hh, _ in placed if hh == h) for h in used_hosts}
    slots = []
    for rank, (h, lr) in enumerate(placed):
        cross_members = [hh for hh in used_hosts if local_sizes[hh] > lr]
        slots.append(Slot(h, rank, lr, local_sizes[h], cross_members.index(h), len(cross_members)))
    return slots


# horovodrun tuning flag -> env var
_TUNING = [
    ("--fusion-threshold-mb", "HOROVOD_FUSION_THRESHOLD", lambda v: str(int(float(v) * 2 ** 20))),
    ("--cycle-time-ms", "HOROVOD_CYCLE_TIME", str),
    ("--cache-capacity", "HOROVOD_CACHE_CAPACITY", str),
    ("--timeline-filename", "HOROVOD_TIMELINE", str),
    ("--autotune-log-file", "HOROVOD_AUTOTUNE_LOG", str),
    ("--stall-check-warning-time-seconds", "HOROVOD_STALL_CHECK_TIME_SECONDS", str),
    ("--stall-check-shutdown-time-seconds", "HOROVOD_STALL_SHUTDOWN_TIME_SECONDS", str),
    ("--log-level", "HOROVOD_LOG_LEVEL", str),
    ("--bucket-mb", "MIVOD_BUCKET_MB", str),
    ("--first-bucket-mb", "MIVOD_FIRST_BUCKET_MB", str),
    ("--transport", "MIVOD_TRANSPORT", str),
]
_TUNING_BOOL = [
    ("--hierarchical-allreduce", "HOROVOD_HIERARCHICAL_ALLREDUCE"),
    ("--hierarchical-allgather", "HOROVOD_HIERARCHICAL_ALLGATHER"),
    ("--timeline-mark-cycles", "HOROVOD_TIMELINE_MARK_CYCLES"),
    ("--autotune", "HOROVOD_AUTOTUNE"),
    ("--no-stall-check", "HOROVOD_STALL_CHECK_DISABLE"),
    ("--log-hide-timestamp", "HOROVOD_LOG_HIDE_TIME"),
]


def build_parser() -> argparse.ArgumentParser:
    p = argparse.ArgumentParser(prog="mivodrun", description=__doc__.split("\n")[0],
                                allow_abbrev=False)
    p.add_argument("-np", "--num-proc", "-n", dest="np", type=int, default=None)
    p.add_argument("-H", "--hosts", "-host", dest="hosts", default=None)
    p.add_argument("--hostfile", "-hostfile", "--machinefile", dest="hostfile", default=None)
    p.add_argument("-x", dest="export", action="append", default=[],
                   help="export VAR (or VAR=value) to every rank (mpirun -x)")
    p.add_argument("--tag-output", "-tag-output", dest="tag_output", action="store_true")
    p.add_argument("--verbose", "-v", action="store_true")
    p.add_argument("--start-timeout", type=float, default=600.0)
    p.add_argument("--master-port", type=int, default=0)
    p.add_argument("--ssh-port", type=int, default=None)
    p.add_argument("--network-interface", default=None)
    p.add_argument("--check-build", action="store_true",
                   help="print the frameworks / controllers / tensor ops this install provides")
    p.add_argument("--config-file", default=None, help="horovodrun YAML config file")
    p.add_argument("--output-filename", default=None,
                   help="also write each rank's output to DIR/rank.N/{stdout,stderr}")
    p.add_argument("--disable-cache", action="store_true",
                   help="disable the coordinator response cache (HOROVOD_CACHE_CAPACITY=0)")
    p.add_argument("--gloo", action="store_true", help="accepted for horovodrun parity")
    p.add_argument("--mpi", action="store_true", help="accepted; mivod never uses MPI")
    # mpirun flags accepted and ignored
    p.add_argument("-bind-to", "--bind-to", dest="bind_to", default=None)
    p.add_argument("-map-by", "--map-by", dest="map_by", default=None)
    p.add_argument("-mca", "--mca", dest="mca", nargs=2, action="append", default=[])
    p.add_argument("--allow-run-as-root", "-allow-run-as-root", action="store_true")
    p.add_argument("--oversubscribe", "-oversubscribe", action="store_true")
    for flag, _env, _conv in _TUNING:
        p.add_argument(flag, default=None)
    for flag, _env in _TUNING_BOOL:
        p.add_argument(flag, action="store_true")
    p.add_argument("command", nargs=argparse.REMAINDER)
    return p


def tuning_env(args) -> Dict[str, str]:
    env = {}
    for flag, var, conv in _TUNING:
        v = getattr(args, flag.lstrip("-").replace("-", "_"))
        if v is not None:
            env[var] = conv(v)
    for flag, var in _TUNING_BOOL:
        if getattr(args, flag.lstrip("-").replace("-", "_")):
            env[var] = "1"
    return env


# horovodrun --config-file sections -> (flag attribute, env var, converter)
_CONFIG_KEYS = {
    ("params", "fusion_threshold_mb"): ("HOROVOD_FUSION_THRESHOLD", lambda v: str(int(float(v) * 2 ** 20))),
    ("params", "cycle_time_ms"): ("HOROVOD_CYCLE_TIME", str),
    ("params", "cache_capacity"): ("HOROVOD_CACHE_CAPACITY", str),
    ("params", "hierarchical_allreduce"): ("HOROVOD_HIERARCHICAL_ALLREDUCE", lambda v: "1" if v else "0"),
    ("params", "hierarchical_allgather"): ("HOROVOD_HIERARCHICAL_ALLGATHER", lambda v: "1" if v else "0"),
    ("autotune", "enabled"): ("HOROVOD_AUTOTUNE", lambda v: "1" if v else "0"),
    ("autotune", "log_file"): ("HOROVOD_AUTOTUNE_LOG", str),
    ("timeline", "filename"): ("HOROVOD_TIMELINE", str),
    ("timeline", "mark_cycles"): ("HOROVOD_TIMELINE_MARK_CYCLES", lambda v: "1" if v else "0"),
    ("stall_check", "enabled"): ("HOROVOD_STALL_CHECK_DISABLE", lambda v: "0" if v else "1"),
    ("stall_check", "warning_time_seconds"): ("HOROVOD_STALL_CHECK_TIME_SECONDS", str),
    ("stall_check", "shutdown_time_seconds"): ("HOROVOD_STALL_SHUTDOWN_TIME_SECONDS", str),
    ("logging", "level"): ("HOROVOD_LOG_LEVEL", str),
    ("logging", "hide_timestamp"): ("HOROVOD_LOG_HIDE_TIME", lambda v: "1" if v else "0"),
    ("mivod", "bucket_mb"): ("MIVOD_BUCKET_MB", str),
    ("mivod", "first_bucket_mb"): ("MIVOD_FIRST_BUCKET_MB", str),
}


def config_file_env(path: str) -> Dict[str, str]:
    """Env for a horovodrun ``--config-file`` (YAML, safe loader)."""
    import yaml
    with open(path) as f:
        cfg = yaml.safe_load(f) or {}
    if not isinstance(cfg, dict):
        raise ValueError(f"{path}: top level must be a mapping")
    env = {}
    for section, body in cfg.items():
        if not isinstance(body, dict):
            raise ValueError(f"{path}: section {section!r} must be a mapping")
        for key, val in body.items():
            ent = _CONFIG_KEYS.get((section, key))
            if ent is None:
                raise ValueError(f"{path}: unknown setting {section}.{key}")
            env[ent[0]] = ent[1](val)
    return env


def check_build() -> str:
    """horovodrun --check-build equivalent: what this mivod install provides."""
    def probe(mod):
        try:
            __import__(mod)
            return True
        except Exception:
            return False

    def box(ok):
        return "[X]" if ok else "[ ]"

    import torch
    dist = probe("torch.distributed")
    rccl = dist and torch.distributed.is_nccl_available() and torch.version.hip is not None
    gloo = dist and torch.distributed.is_gloo_available()
    lines = ["mivod (Horovod API on MI355X)", "",
             "Available Frameworks:",
             f"    {box(True)} PyTorch ({torch.__version__})",
             f"    {box(probe('mivod.kerasfw'))} Keras (mivod.kerasfw on PyTorch)",
             f"    {box(False)} TensorFlow", f"    {box(False)} MXNet", "",
             "Available Controllers:",
             f"    {box(probe('mivod._mvcore'))} TCP coordinator (mivod._mvcore, C++)",
             f"    {box(False)} MPI", f"    {box(gloo)} Gloo", "",
             "Available Tensor Operations:",
             f"    {box(rccl)} RCCL (xGMI)", f"    {box(False)} NCCL", f"    {box(False)} DDL",
             f"    {box(False)} CCL", f"    {box(False)} MPI", f"    {box(gloo)} Gloo",
             f"    {box(probe('mivod._mvk'))} gfx950 HIP kernels (mivod._mvk)"]
    return "\n".join(lines)


def exported_env(exports: Sequence[str]) -> Dict[str, str]:
    env = {}
    for e in exports:
        if "=" in e:
            k, v = e.split("=", 1)
            env[k] = v
        elif e in os.environ:
            env[e] = os.environ[e]
    return env


def rank_env(slot: Slot, size: int, master_addr: str, master_port: int,
             store_port: int = 0) -> Dict[str, str]:
    env = {
        "HOROVOD_RANK": str(slot.rank), "HOROVOD_SIZE": str(size),
        "HOROVOD_LOCAL_RANK": str(slot.local_rank), "HOROVOD_LOCAL_SIZE": str(slot.local_size),
        "HOROVOD_CROSS_RANK": str(slot.cross_rank), "HOROVOD_CROSS_SIZE": str(slot.cross_size),
        "HOROVOD_HOSTNAME": slot.host,
        "RANK": str(slot.rank), "WORLD_SIZE": str(size), "LOCAL_RANK": str(slot.local_rank),
        "LOCAL_WORLD_SIZE": str(slot.local_size), "GROUP_RANK": str(slot.cross_rank),
        "MASTER_ADDR": master_addr, "MASTER_PORT": str(master_port),
        "HSA_ENABLE_IPC_MODE_LEGACY": os.environ.get("HSA_ENABLE_IPC_MODE_LEGACY", "0"),
    }
    if store_port:
        # the launcher-hosted native rendezvous store (csrc/engine/store.cc), under
        # horovodrun's Gloo rendezvous variable names
        env["HOROVOD_GLOO_RENDEZVOUS_ADDR"] = master_addr
        env["HOROVOD_GLOO_RENDEZVOUS_PORT"] = str(store_port)
    return env


def _is_local(host: str) -> bool:
    if host in LOCAL_NAMES:
        return True
    try:
        return host in (socket.gethostname(), socket.getfqdn())
    except Exception:
        return False


def _free_port() -> int:
    s = socket.socket()
    s.bind(("", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def ssh_command(host: str, env: Dict[str, str], command: List[str], cwd: str,
                ssh_port: Optional[int] = None) -> List[str]:
    exports = " ".join(f"{k}={shlex.quote(v)}" for k, v in sorted(env.items()))
    remote = f"cd {shlex.quote(cwd)} && env {exports} {' '.join(shlex.quote(c) for c in command)}"
    cmd = ["ssh", "-o", "StrictHostKeyChecking=no", "-o", "BatchMode=yes"]
    if ssh_port:
        cmd += ["-p", str(ssh_port)]
    return cmd + [host, remote]


class _Pump(threading.Thread):
    def __init__(self, stream, out, prefix: str, copy_path: Optional[str] = None):
        super().__init__(daemon=True)
        self.stream, self.out, self.prefix, self.copy_path = stream, out, prefix, copy_path

    def run(self):
        copy = open(self.copy_path, "w") if self.copy_path else None
        try:
            for line in iter(self.stream.readline, b""):
                text = line.decode(errors="replace")
                self.out.write(self.prefix + text if self.prefix else text)
                self.out.flush()
                if copy:
                    copy.write(text)
                    copy.flush()
        finally:
            if copy:
                copy.close()


def launch(slots: List[Slot], command: List[str], extra_env: Dict[str, str],
           tag_output: Optional[bool] = None, master_port: int = 0,
           ssh_port: Optional[int] = None,
           verbose: bool = False, output_dir: Optional[str] = None) -> int:
    size = len(slots)
    first = slots[0].host
    master_addr = "127.0.0.1" if _is_local(first) else first
    if all(_is_local(s.host) for s in slots):
        master_addr = "127.0.0.1"
    master_port = master_port or _free_port()
    server = None
    store_port = 0
    if os.environ.get("MIVOD_STORE", "native") != "torch":
        try:
            from .store import serve
            server = serve("127.0.0.1" if master_addr == "127.0.0.1" else "0.0.0.0", 0)
            store_port = server.port
        except Exception as e:     # no native core: ranks fall back to torch's TCPStore
            if verbose:
                print(f"[mivodrun] native rendezvous store unavailable ({e}); using "
                      "torch's TCPStore", file=sys.stderr)
    procs: List[subprocess.Popen] = []
    pumps = []
    tag = tag_output if tag_output is not None else size > 1   # default: tag when N > 1
    cwd = os.getcwd()
    for s in slots:
        env = dict(os.environ)
        env.update(extra_env)
        env.update(rank_env(s, size, master_addr, master_port, store_port))
        if _is_local(s.host):
            cmd, penv = command, env
        else:
            renv = dict(extra_env)
            renv.update(rank_env(s, size, master_addr, master_port, store_port))
            cmd, penv = ssh_command(s.host, renv, command, cwd, ssh_port), dict(os.environ)
        if verbose:
            print(f"[mivodrun] rank {s.rank} on {s.host}: {' '.join(cmd)}", file=sys.stderr)
        p = subprocess.Popen(cmd, env=penv, stdout=subprocess.PIPE, stderr=subprocess.PIPE,
                             start_new_session=True)
        procs.append(p)
        pre_o = f"[{s.rank}]<stdout>:" if tag else ""
        pre_e = f"[{s.rank}]<stderr>:" if tag else ""
        rdir = None
        if output_dir:
            rdir = os.path.join(output_dir, f"rank.{s.rank}")
            os.makedirs(rdir, exist_ok=True)
        for st, out, pre, nm in ((p.stdout, sys.stdout, pre_o, "stdout"),
                                 (p.stderr, sys.stderr, pre_e, "stderr")):
            t = _Pump(st, out, pre, os.path.join(rdir, nm) if rdir else None)
            t.start()
            pumps.append(t)

    def terminate_all(sig=signal.SIGTERM):
        for p in procs:
            if p.poll() is None:
                try:
                    os.killpg(p.pid, sig)
                except ProcessLookupError:
                    pass

    def on_signal(signum, _frame):
        terminate_all(signal.SIGTERM)

    old_int = signal.signal(signal.SIGINT, on_signal)
    old_term = signal.signal(signal.SIGTERM, on_signal)
    rc = 0
    try:
        remaining = set(range(size))
        while remaining:
            for i in list(remaining):
                r = procs[i].poll()
                if r is None:
                    continue
                remaining.discard(i)
                if r != 0 and rc == 0:
                    rc = r if r > 0 else 128 - r
                    print(f"[mivodrun] rank {slots[i].rank} exited with code {r}; terminating "
                          f"the remaining ranks", file=sys.stderr)
                    terminate_all(signal.SIGTERM)
                    deadline = time.time() + 10
                    while time.time() < deadline and any(p.poll() is None for p in procs):
                        time.sleep(0.1)
                    terminate_all(signal.SIGKILL)
            time.sleep(0.05)
    finally:
        signal.signal(signal.SIGINT, old_int)
        signal.signal(signal.SIGTERM, old_term)
        for t in pumps:
            t.join(timeout=5)
        if server is not None:
            server.close()
    return rc


def main(argv: Optional[List[str]] = None) -> int:
    args = build_parser().parse_args(argv)
    if args.check_build:
        print(check_build())
        return 0
    command = list(args.command)
    if command and command[0] == "--":
        command = command[1:]
    if not command:
        build_parser().error("no command given")
    if args.hostfile:
        hosts = parse_hostfile(args.hostfile)
    elif args.hosts:
        hosts = parse_hosts(args.hosts)
    else:
        hosts = [("localhost", args.np or 1)]
    np = args.np or sum(n for _, n in hosts)
    slots = assign_slots(hosts, np)
    env = config_file_env(args.config_file) if args.config_file else {}
    env.update(tuning_env(args))                  # command-line flags win over the file
    if args.disable_cache:
        env["HOROVOD_CACHE_CAPACITY"] = "0"
    if args.network_interface:
        env["NCCL_SOCKET_IFNAME"] = args.network_interface
        env["GLOO_SOCKET_IFNAME"] = args.network_interface
    env.update(exported_env(args.export))
    return launch(slots, command, env, args.tag_output or None, args.master_port, args.ssh_port,
                  args.verbose, args.output_filename)


if __name__ == "__main__":
    sys.exit(main())
