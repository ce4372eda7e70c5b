"""HBM traffic per launch of the pass kernel, from rocprofv3 PMC runs -> a JSON that
bench.py --traffic-json reads (only when it names the same config and size).

usage: python tools/bench_pmc.py TAG CONFIG N OUT.json [KERNEL]
  gpurun_out/TAG_fetch, TAG_write          FETCH_SIZE / WRITE_SIZE runs of bench.py (one
                                           counter per rocprofv3 run, MI355X_MICROARCH.md HBM)
  gpurun_out/TAG_cfetch, TAG_cwrite        the same counters over the calibration kernel
                                           (tools/lab2.py --emu 1024:36:0: the pass's exact
                                           load/store instructions, contiguous, known bytes)

MI355X_MICROARCH.md: FETCH_SIZE reads 1/2 of the bytes of a 16-B/lane streaming read; other
widths are uncalibrated.  The pass loads 4 B/lane (global_load_dword) and stores 4 B/lane, so
the correction factors are measured here on the calibration kernel, which moves exactly
2^27 x 4 B each way: factor = known bytes / counter bytes.
"""
import csv
import glob
import json
import os
import statistics
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def per_launch(tag_dir: str, counter: str, name_part: str) -> float:
    vals = []
    for path in glob.glob(os.path.join(REPO, "gpurun_out", tag_dir, "**", "*counter_collection.csv"),
                          recursive=True):
        for r in csv.DictReader(open(path)):
            if name_part in r["Kernel_Name"] and r["Counter_Name"] == counter:
                vals.append(float(r["Counter_Value"]))
    if not vals:
        raise SystemExit(f"no {counter} rows for {name_part} under gpurun_out/{tag_dir}")
    return statistics.mean(vals) * 1024.0   # KiB -> bytes


def main():
    tag, config, n, out_path = sys.argv[1], sys.argv[2], int(sys.argv[3]), sys.argv[4]
    kern = sys.argv[5] if len(sys.argv) > 5 else "grs_onesweep_v4"
    fetch = per_launch(f"{tag}_fetch", "FETCH_SIZE", kern)
    write = per_launch(f"{tag}_write", "WRITE_SIZE", kern)
    known = (1 << 27) * 4
    cf = known / per_launch(f"{tag}_cfetch", "FETCH_SIZE", "scatter_emu")
    cw = known / per_launch(f"{tag}_cwrite", "WRITE_SIZE", "scatter_emu")
    rec = {"config": config, "n": n,
           "hbm_bytes_per_launch": round(cf * fetch + cw * write),
           "read_bytes": round(cf * fetch), "write_bytes": round(cw * write),
           "fetch_size_raw": round(fetch), "write_size_raw": round(write),
           "read_factor": round(cf, 4), "write_factor": round(cw, 4),
           "algorithmic_bytes_per_launch": n * 8,
           "source": f"rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE over bench.py --config {config} "
                     f"and the calibration kernel ({tag})"}
    json.dump(rec, open(out_path, "w"), indent=1)
    print(json.dumps(rec))


if __name__ == "__main__":
    main()
