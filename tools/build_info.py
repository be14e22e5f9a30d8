#!/usr/bin/env python3
"""Provenance of a built library (written next to it by the Makefile as build_info.json, travels to the GPU box
with the tree): the git commit it was built from, whether the tracked sources differed from that commit, and the
library's sha256 -- so a measurement (bench.py, tools/pmc_summary.py) can say which build it timed.
    python tools/build_info.py sp-slam_amd/libspslam_gpu.so"""
import datetime
import hashlib
import json
import pathlib
import subprocess
import sys

ROOT = pathlib.Path(__file__).resolve().parents[1]


def lib_sha256(path):
    return hashlib.sha256(pathlib.Path(path).read_bytes()).hexdigest()


def git(*args):
    try:
        return subprocess.run(["git", "-C", str(ROOT), *args], capture_output=True, text=True, timeout=20).stdout.strip()
    except (OSError, subprocess.SubprocessError):
        return ""


def info(lib):
    dirty = git("status", "--porcelain", "--untracked-files=no", "--", "sp-slam_amd/csrc", "include")
    return {"git_head": git("rev-parse", "HEAD") or "unknown", "sources_dirty": bool(dirty),
            "lib": str(pathlib.Path(lib).resolve().relative_to(ROOT)), "lib_sha256": lib_sha256(lib),
            "built_utc": datetime.datetime.utcnow().isoformat(timespec="seconds")}


if __name__ == "__main__":
    print(json.dumps(info(sys.argv[1]), indent=1))
