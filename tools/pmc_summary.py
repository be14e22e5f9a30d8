#!/usr/bin/env python3
"""HBM traffic per launch from two rocprofv3 PMC passes (tools/pmc_round.sh).

    python tools/pmc_summary.py gpurun_out/pmc_fetch_c2 gpurun_out/pmc_write_c2 profiles/pmc_c2_b256.json

FETCH_SIZE / WRITE_SIZE are kilobytes per dispatch.  MI355X_MICROARCH.md
("HBM"): on gfx950 FETCH_SIZE reports half the bytes of wide coalesced
streaming reads, so fetch bytes = 2 x FETCH_SIZE x 1024 (the correction is
calibrated for 16 B/lane streaming loads; narrower gathers are uncalibrated);
WRITE_SIZE is taken as is.  Output: {kernel: traffic bytes per timed launch of that kernel kind (bench.py)} plus
a "detail" map with the two components and the dispatch count.
"""
import collections
import csv
import json
import re
import sys


# kernel function names that bench.py times under another kind name
ALIAS = {"grab_vec_kernel": "grab_rgbd_kernel", "grab_scalar_kernel": "grab_rgbd_kernel"}


def short(name):
    m = re.search(r"(\w+_kernel)\b", name)
    k = m.group(1) if m else name.split("(")[0][-60:]
    return ALIAS.get(k, k)


def load(d, counter):
    path = f"{d}/run_counter_collection.csv"
    acc = collections.defaultdict(list)
    with open(path) as f:
        for row in csv.DictReader(f):
            if row["Counter_Name"] == counter:
                acc[short(row["Kernel_Name"])].append(float(row["Counter_Value"]))
    return acc


# dispatches per timed kernel-kind launch in bench.py (the level kind times its 8 per-level launches together)
PER_KIND = {"level_kernel": 8}


def sized_reads(d):
    """Read bytes per dispatch from the size-resolved memory-side request counters (one pass of
    TCC_EA0_RDREQ{,_32B,_64B,_128B}_sum): 32 n32 + 64 n64 + 128 n128, the requests' own sizes, instead of
    FETCH_SIZE's 64 B per request (uncalibrated for narrow gathers, MI355X_MICROARCH.md "HBM")."""
    c = {n: load(d, f"TCC_EA0_RDREQ{n}_sum") for n in ("", "_32B", "_64B", "_128B")}
    out = {}
    for k, tot in c[""].items():
        n32, n64, n128 = (c[n].get(k, [0] * len(tot)) for n in ("_32B", "_64B", "_128B"))
        out[k] = dict(req=sum(tot), n32=sum(n32), n64=sum(n64), n128=sum(n128),
                      bytes=[32 * a + 64 * b + 128 * e for a, b, e in zip(n32, n64, n128)])
    return out


def main(fetch_dir, write_dir, out, sized_dir=None):
    fe, wr = load(fetch_dir, "FETCH_SIZE"), load(write_dir, "WRITE_SIZE")
    sz = sized_reads(sized_dir) if sized_dir else {}
    res, detail = {}, {}
    for k in sorted(set(fe) | set(wr)):
        if not k.endswith("_kernel"):
            continue
        per = PER_KIND.get(k, 1)
        f = sum(fe.get(k, [0])) / max(len(fe.get(k, [])) / per, 1) * 1024 * 2
        w = sum(wr.get(k, [0])) / max(len(wr.get(k, [])) / per, 1) * 1024
        detail[k] = dict(fetch_bytes=f, write_bytes=w, dispatches=len(fe.get(k, [])))
        if k in sz:  # size-resolved read bytes replace 2 x FETCH_SIZE
            q = sz[k]
            f = sum(q["bytes"]) / max(len(q["bytes"]) / per, 1)
            detail[k].update(read_bytes_sized=f, fetch_size_x2=detail[k]["fetch_bytes"], rdreq=q["req"],
                             rdreq_32b=q["n32"], rdreq_64b=q["n64"], rdreq_128b=q["n128"])
            detail[k]["fetch_bytes"] = f
        res[k] = f + w
        print(f"{k:28s} fetch {f / 1e6:10.3f} MB  write {w / 1e6:10.3f} MB  per launch  ({len(fe.get(k, []))} launches)")
    res["detail"] = detail
    import datetime
    import os
    import pathlib
    root = pathlib.Path(__file__).resolve().parents[1]
    bi = root / "sp-slam_amd" / "build_info.json"
    build = json.loads(bi.read_text()) if bi.exists() else {}
    sys.path.insert(0, str(root / "tools"))
    import build_info
    res["provenance"] = {"measured_utc": datetime.datetime.utcnow().isoformat(timespec="seconds"),
                         "git_head": build.get("git_head", os.environ.get("SPSLAM_GIT_HEAD", "unknown")),
                         "sources_dirty": build.get("sources_dirty"),
                         "lib_sha256": build_info.lib_sha256(root / "sp-slam_amd" / "libspslam_gpu.so"),
                         "command": os.environ.get("SPSLAM_PMC_CMD", "tools/pmc_round.sh")}
    res["note"] = (("HBM bytes per launch = read bytes from the size-resolved TCC_EA0_RDREQ_{32B,64B,128B} request "
                    "counts (detail: read_bytes_sized; 2 x FETCH_SIZE kept as fetch_size_x2) + WRITE_SIZE"
                    if sz else "HBM bytes per launch = 2 x FETCH_SIZE + WRITE_SIZE (KB x 1024)") +
                   ", rocprofv3 separate --pmc passes, gfx950 corrections per MI355X_MICROARCH.md")
    with open(out, "w") as fo:
        json.dump(res, fo, indent=1)


if __name__ == "__main__":
    main(*sys.argv[1:5])
