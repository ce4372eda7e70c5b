"""HBM traffic of the pass kernel from rocprofv3 PMC runs of bench.py -> profiles/pmc_traffic.json.

usage: python tools/bench_pmc.py TAG CONFIG N
  reads gpurun_out/TAG_fetch/**/*counter_collection.csv and gpurun_out/TAG_write/... (one
  counter per rocprofv3 run, as MI355X_MICROARCH.md's HBM section prescribes) and records the
  mean bytes per launch of the onesweep pass kernel.

FETCH_SIZE and WRITE_SIZE are in KiB.  gfx950 correction (MI355X_MICROARCH.md, HBM section):
FETCH_SIZE reports half of the bytes of a wide (16 B/lane) coalesced streaming read, which is
how the pass reads its keys (global_load_lds_dwordx4), so fetched bytes = 2 x FETCH_SIZE;
WRITE_SIZE is exact for streaming stores.
"""
import csv
import glob
import json
import os
import statistics
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def per_launch(tag_dir: str, counter: str) -> float:
    vals = []
    for path in glob.glob(os.path.join(REPO, "gpurun_out", tag_dir, "**", "*counter_collection.csv"),
                          recursive=True):
        for r in csv.DictReader(open(path)):
            if "onesweep" in r["Kernel_Name"] and r["Counter_Name"] == counter:
                vals.append(float(r["Counter_Value"]))
    if not vals:
        raise SystemExit(f"no {counter} rows for an onesweep kernel under gpurun_out/{tag_dir}")
    return statistics.mean(vals) * 1024.0


def main():
    tag, config, n = sys.argv[1], sys.argv[2], int(sys.argv[3])
    fetch = per_launch(f"{tag}_fetch", "FETCH_SIZE")
    write = per_launch(f"{tag}_write", "WRITE_SIZE")
    out_path = os.path.join(REPO, "profiles", "pmc_traffic.json")
    db = json.load(open(out_path)) if os.path.exists(out_path) else {}
    db[f"{config}:{n}"] = {
        "hbm_bytes_per_launch": round(2 * fetch + write),
        "fetch_size_bytes_raw": round(fetch), "write_size_bytes": round(write),
        "correction": "fetched = 2 x FETCH_SIZE (gfx950 16-B/lane streaming reads), WRITE_SIZE exact",
        "source": f"rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE runs of bench.py --config {config} ({tag})",
    }
    json.dump(db, open(out_path, "w"), indent=1)
    # the box's profiles/ does not travel back: a copy under gpurun_out/ is merged home
    os.makedirs(os.path.join(REPO, "gpurun_out"), exist_ok=True)
    json.dump(db, open(os.path.join(REPO, "gpurun_out", "pmc_traffic.json"), "w"), indent=1)
    print(json.dumps(db[f"{config}:{n}"]))


if __name__ == "__main__":
    main()
