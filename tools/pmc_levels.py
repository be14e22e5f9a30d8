#!/usr/bin/env python3
"""level_kernel traffic per pyramid level against its algorithmic bytes, with the FETCH_SIZE scale calibrated
per load width (tools/fetch_probe.hip).  Inputs: three rocprofv3 --pmc directories (tools/pmc_levels.sh).

    python tools/pmc_levels.py gpurun_out/probe_fetch gpurun_out/lv_fetch gpurun_out/lv_write [B]

Level l's dispatch is recognised by its grid (tiles(l) x B workgroups of 256 threads).  Algorithmic bytes per
frame: reads = the level below (the input gray frame at level 0), writes = level image (l > 0) + blurred
image + FAST score map, all u8 w x h."""
import collections
import csv
import json
import pathlib
import sys

ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))


def rows(d, counter):
    with open(f"{d}/run_counter_collection.csv") as f:
        return [r for r in csv.DictReader(f) if r["Counter_Name"] == counter]


def main(probe, fdir, wdir, B=256):
    import bench
    out = {"probe": {}, "levels": []}
    per = collections.defaultdict(list)
    for r in rows(probe, "FETCH_SIZE"):
        per[r["Kernel_Name"].split("(")[0]].append(float(r["Counter_Value"]) * 1024)
    true = 256 << 20
    for k, v in sorted(per.items()):
        out["probe"][k] = {"fetch_size_bytes": sum(v) / len(v), "scale_vs_true": sum(v) / len(v) / true}
        print(f"probe {k:10s} FETCH_SIZE {sum(v) / len(v) / 1e6:9.2f} MB per dispatch, x{true / (sum(v) / len(v)):.3f} "
              f"to the true 268.44 MB")
    sizes = bench.level_sizes(640, 480)
    tiles = [(-(-w // 64)) * (-(-h // 32)) for w, h in sizes]
    grid_to_level = {t * B * 256: l for l, t in enumerate(tiles)}
    fe, wr = collections.defaultdict(list), collections.defaultdict(list)
    for r in rows(fdir, "FETCH_SIZE"):
        if "level_kernel" in r["Kernel_Name"]:
            fe[grid_to_level.get(int(r["Grid_Size"]), -1)].append(float(r["Counter_Value"]) * 1024)
    for r in rows(wdir, "WRITE_SIZE"):
        if "level_kernel" in r["Kernel_Name"]:
            wr[grid_to_level.get(int(r["Grid_Size"]), -1)].append(float(r["Counter_Value"]) * 1024)
    s4 = out["probe"].get("probe4", {}).get("scale_vs_true")
    print(f"{'level':>5} {'w x h':>10} {'alg read':>10} {'FETCH raw':>10} {'raw/alg':>8} {'x2/alg':>7} "
          f"{'dword-cal/alg':>13} {'alg write':>10} {'WRITE':>10} {'w/alg':>6}")
    for l, (w, h) in enumerate(sizes):
        rd = (sizes[l - 1][0] * sizes[l - 1][1] if l else w * h) * B
        wa = (3 if l else 2) * w * h * B
        f = sum(fe[l]) / max(len(fe[l]), 1)
        wb = sum(wr[l]) / max(len(wr[l]), 1)
        cal = f / s4 if s4 else None
        rec = {"level": l, "w": w, "h": h, "alg_read": rd, "fetch_raw": f, "alg_write": wa, "write": wb,
               "fetch_dword_calibrated": cal, "dispatches": len(fe[l])}
        out["levels"].append(rec)
        print(f"{l:5d} {w:4d}x{h:<5d} {rd / 1e6:10.2f} {f / 1e6:10.2f} {f / rd:8.2f} {2 * f / rd:7.2f} "
              f"{(cal / rd if cal else float('nan')):13.2f} {wa / 1e6:10.2f} {wb / 1e6:10.2f} {wb / wa:6.2f}")
    return out


if __name__ == "__main__":
    a = sys.argv[1:]
    res = main(a[0], a[1], a[2], int(a[3]) if len(a) > 3 else 256)
    if len(a) > 4:
        pathlib.Path(a[4]).write_text(json.dumps(res, indent=1))
