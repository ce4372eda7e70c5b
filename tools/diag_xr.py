"""XCD-range diagnostics: library sorts at several sizes with xcd_ranges on / off, checked
against torch's sort (u32 keys)."""
import sys
import torch
sys.path.insert(0, ".")
import gpuradixsort_amd as grs

dev = torch.device("cuda", 0)
for n in [int(x) for x in sys.argv[1:]]:
    base = torch.empty(n, dtype=torch.uint32, device=dev)
    grs.fill_splitmix(base, 12345)
    ref = torch.sort(base.view(torch.int32).to(torch.int64) & 0xFFFFFFFF).values
    for xr in ("on", "off"):
        for xl in ("size", "always", "never"):
            s = grs.RadixSorter(n, key_bits=32, options={"xcd_ranges": xr, "xl": xl})
            k = base.clone()
            s.sort(k)
            s.check_error()
            got = k.view(torch.int32).to(torch.int64) & 0xFFFFFFFF
            bad = int((got != ref).sum())
            first = int((got != ref).nonzero()[0]) if bad else -1
            print(f"n={n} xr={xr} xl={xl} kernel={s.pass_kernel_for(n)} mismatches={bad} first={first}", flush=True)
            s.close()
            del k, got
    del base, ref
    torch.cuda.empty_cache()
