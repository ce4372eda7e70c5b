"""Driver of tools/lab6.hip: the partition pass of 2^27 uniform u32 keys into 8 buckets with its
digit computed four ways (see lab6.hip); median kernel time of 9 launches each, outputs checked
against a stable partition by the top 3 bits."""
import ctypes
import os
import statistics
import sys

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
import gpuradixsort_amd as grs  # noqa: E402

L = ctypes.CDLL(os.path.join(HERE, "liblab6.so"))
L.lab6_status_words.restype = ctypes.c_size_t
vp = ctypes.c_void_p


def main():
    dev = torch.device("cuda", 0)
    n = 1 << 27
    keys = torch.empty(n, dtype=torch.int32, device=dev)
    grs.fill_splitmix(keys, 4)
    top = (keys.to(torch.int64) & 0xFFFFFFFF) >> 29
    hist = torch.zeros(16, dtype=torch.int32, device=dev)
    hist[:8] = torch.bincount(top, minlength=8).to(torch.int32)
    want = keys[torch.sort(top, stable=True).indices]
    out = torch.empty_like(keys)
    sw = L.lab6_status_words(n)
    st = torch.zeros(2 * sw, dtype=torch.int32, device=dev)
    tk = torch.zeros(8, dtype=torch.int32, device=dev)
    err = torch.zeros(4, dtype=torch.int32, device=dev)
    lut = torch.full((4096,), 0xFF, dtype=torch.uint8, device=dev)
    p = torch.arange(4096, device=dev)
    # prefix p covers keys [p << 20, (p + 1) << 20): one bucket unless a splitter j << 29 lies
    # strictly inside it (splitters at prefix starts keep the prefix whole)
    lut[:] = (p >> 9).to(torch.uint8)
    stream = vp(torch.cuda.current_stream().cuda_stream)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    modes = [(0, 16, "SplitterIdxDigit (shipped)"), (1, 16, "SplitterDigitN, 32-bit counters"),
             (1, 272, "SplitterDigitN, 16-bit counters"), (2, 16, "top 3 bits, 32-bit counters"),
             (2, 272, "top 3 bits, 16-bit counters"), (3, 16, "12-bit LUT + composite"),
             (8, 16, "compares, no LDS table, 1024x36"), (4, 16, "shipped digit, 1024x32"),
             (7, 16, "compares, no LDS table, 1024x32"), (5, 16, "shipped digit, 1024x28"),
             (6, 16, "shipped digit, 1024x24"), (9, 16, "32-bit compares + tie branch, 1024x32")]
    if len(sys.argv) > 1:
        modes = [m for m in modes if str(m[0]) in sys.argv[1].split(",")]
    for mode, opt, name in modes:
        ts = []
        for rep in range(9):
            st.zero_()
            tk.zero_()
            out.fill_(-1)
            e0.record()
            rc = L.lab6_part(mode, opt, vp(keys.data_ptr()), vp(out.data_ptr()), n, vp(hist.data_ptr()),
                             vp(tk.data_ptr()), vp(st.data_ptr()), vp(st.data_ptr() + 4 * sw),
                             vp(err.data_ptr()), vp(lut.data_ptr()), stream)
            e1.record()
            torch.cuda.synchronize()
            assert rc == 0, (mode, opt, rc)
            ts.append(e0.elapsed_time(e1))
        ok = bool(torch.equal(out, want)) and int(err[0].item()) == 0
        print(f"{name:36s} {statistics.median(ts) * 1e3:8.1f} us  exact={ok}", flush=True)


if __name__ == "__main__":
    main()
