"""Process launch for the multi-GPU bench: one process per GPU, started by a
parent that never touches the GPU itself.

`python3 bench.py --gpus N` is how the driver runs the bench.  Without
WORLD_SIZE in the environment that process is not a rank: it counts the
visible GPUs in a child process, then starts N ranks under
`torch.distributed.run` (RCCL process group per rank, 127.0.0.1 rendezvous)
as a child, and relays rank 0's one JSON line.  Nothing here initialises HIP,
so the parent may start further children (the product's one-process
multi-device leg) and no process execs over a GPU-initialised image.

The reference has no multi-GPU path at all (device selection is commented out,
src/gasal2_ssw.cpp:34); its host-side analogue is main.cpp:557-600 (worker
threads, then a host loop summing AlignmentStatistics).
"""
from __future__ import annotations

import json
import os
import socket
import subprocess
import sys


def free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def visible_gpus(timeout: float = 300.0) -> int:
    """GPUs a child process sees (torch.cuda.device_count()), 0 when none or on error.
    Counted in a child so that this process stays free of any HIP state."""
    code = "import torch; print(torch.cuda.device_count() if torch.cuda.is_available() else 0)"
    try:
        p = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=timeout)
    except (OSError, subprocess.TimeoutExpired):
        return 0
    try:
        return int(p.stdout.strip().splitlines()[-1])
    except (ValueError, IndexError):
        return 0


def _relay(cmd: list, env: dict | None, timeout: float | None = None) -> tuple[int, dict | None]:
    """Run `cmd`; stderr passes through live; stdout lines are relayed to stderr
    except the last JSON object line, which is returned parsed.  With `timeout`
    (seconds) the child's process group is killed when it runs longer (exit code
    124, as timeout(1) reports it)."""
    import signal
    import threading
    line = None
    expired = threading.Event()
    with subprocess.Popen(cmd, stdout=subprocess.PIPE, env=env, text=True, bufsize=1,
                          start_new_session=timeout is not None) as p:
        def kill():
            expired.set()
            print(f"[launch] {cmd[1:3]} still running after {timeout:.0f} s: killed", file=sys.stderr, flush=True)
            try:
                os.killpg(p.pid, signal.SIGTERM)
            except OSError:
                return
            try:
                p.wait(timeout=30)
            except subprocess.TimeoutExpired:
                try:
                    os.killpg(p.pid, signal.SIGKILL)
                except OSError:
                    pass
        timer = threading.Timer(timeout, kill) if timeout else None
        if timer:
            timer.daemon = True
            timer.start()
        try:
            for raw in p.stdout:
                s = raw.strip()
                if s.startswith("{") and s.endswith("}"):
                    try:
                        line = json.loads(s)
                        continue
                    except ValueError:
                        pass
                print(raw, end="", file=sys.stderr, flush=True)
            rc = p.wait()
        finally:
            if timer:
                timer.cancel()
    return (124 if expired.is_set() else rc), (None if expired.is_set() else line)


def run_ranks(script: str, script_args: list, nproc: int, env: dict | None = None,
              port: int | None = None) -> tuple[int, dict | None]:
    """`script script_args` as `nproc` ranks of one node under torch.distributed.run.
    Returns (exit code, rank 0's JSON line or None)."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={nproc}",
           "--master-addr=127.0.0.1", f"--master-port={port or free_port()}", script, *script_args]
    return _relay(cmd, env)


def run_child(cmd: list, env: dict | None = None, timeout: float | None = None) -> tuple[int, dict | None]:
    """One more process (e.g. the product's multi-device leg); (exit code, its JSON line).
    `timeout`: kill it (and report 124) after that many seconds."""
    return _relay(cmd, env, timeout)
