"""``--profile`` (Config.profile): re-run the entry point under rocprofv3.

The process that parsed ``--profile`` has not touched the GPU yet; it starts ONE child
``rocprofv3 --kernel-trace --stats -d DIR -o run -- <python> <same entry point + args>`` (the
program directly after ``--``: no shell or env hop, since the profiler's preloaded library
initialises the GPU before the program starts), waits for it, prints the top kernels of the
stats CSV and exits with the child's status. The child sees ``FDX_PROFILE_CHILD=1`` and runs
normally. Counters (``--pmc``) are a separate, manual pass (bench/pmc_gbdt.sh): they must not be
combined with trace domains.
"""
from __future__ import annotations

import csv
import glob
import os
import shutil
import subprocess
import sys
from typing import Optional, Sequence

CHILD_ENV = "FDX_PROFILE_CHILD"


def _strip_profile(argv: Sequence[str]) -> list:
    return [a for a in argv if a not in ("--profile", "--no-profile")]


def child_command(argv: Sequence[str], out_dir: str, module: Optional[str] = None,
                  rocprof: Optional[str] = None) -> list:
    """The child's command line: rocprofv3 with kernel trace + stats, then this interpreter
    running ``module`` (``-m``) or the current script with ``argv`` minus ``--profile``."""
    rocprof = rocprof or shutil.which("rocprofv3") or "/opt/rocm/bin/rocprofv3"
    target = [sys.executable, "-m", module] if module else [sys.executable, os.path.abspath(sys.argv[0])]
    return [rocprof, "--kernel-trace", "--stats", "-d", out_dir, "-o", "run", "--", *target, *_strip_profile(argv)]


def kernel_stats(out_dir: str, top: int = 15) -> list:
    """(name, calls, total ms, percent) of the ``top`` kernels in the run's ``*kernel_stats.csv``."""
    files = sorted(glob.glob(os.path.join(out_dir, "**", "*kernel_stats.csv"), recursive=True))
    rows = []
    for f in files:
        with open(f, newline="") as fh:
            for r in csv.DictReader(fh):
                try:
                    rows.append((r["Name"], int(r["Calls"]), float(r["TotalDurationNs"]) / 1e6,
                                 float(r.get("Percentage", 0.0))))
                except (KeyError, ValueError):
                    continue
    rows.sort(key=lambda t: -t[2])
    return rows[:top]


def run_profiled_if_requested(profile: bool, argv: Optional[Sequence[str]] = None, module: Optional[str] = None,
                              out_dir: Optional[str] = None) -> None:
    """No-op unless ``profile`` is set and this is not already the profiled child; otherwise runs
    the child under rocprofv3 and exits with its status (never returns)."""
    if not profile or os.environ.get(CHILD_ENV):
        return
    argv = list(sys.argv[1:] if argv is None else argv)
    out_dir = out_dir or os.environ.get("FDX_PROFILE_DIR", os.path.join("gpurun_out", "profile"))
    os.makedirs(out_dir, exist_ok=True)
    cmd = child_command(argv, out_dir, module)
    if not (os.path.isfile(cmd[0]) or shutil.which(cmd[0])):
        raise RuntimeError(f"--profile needs rocprofv3 (not found: {cmd[0]})")
    env = dict(os.environ)
    env[CHILD_ENV] = "1"
    env.setdefault("TMPDIR", "/tmp")
    print(f"[profile] {' '.join(cmd)}", file=sys.stderr, flush=True)
    rc = subprocess.call(cmd, env=env)
    for name, calls, ms, pct in kernel_stats(out_dir):
        print(f"[profile] {ms:10.3f} ms {calls:7d} calls {pct:6.2f} %  {name[:110]}", file=sys.stderr)
    print(f"[profile] traces and stats under {out_dir}", file=sys.stderr, flush=True)
    sys.exit(rc)
