"""Driver of tools/barrier_probe.hip: microseconds per round of (stores + grid barrier) in one
persistent launch, per barrier mode, against one launch per round (the kernel boundary)."""
import ctypes
import os
import statistics

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
L = ctypes.CDLL(os.path.join(HERE, "libbarrier_probe.so"))
vp = ctypes.c_void_p


def main():
    dev = torch.device("cuda", 0)
    grid = torch.cuda.get_device_properties(0).multi_processor_count
    rounds = 8
    stream = vp(torch.cuda.current_stream().cuda_stream)
    err = torch.zeros(1, dtype=torch.int32, device=dev)
    ctl = torch.zeros(64, dtype=torch.int32, device=dev)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for words in (16384, 65536):   # 64 KB / 256 KB per workgroup per round (16 / 64 MB in all)
        out = torch.empty(grid * words, dtype=torch.int32, device=dev)

        def timed(fn, reps=7):
            fn()
            torch.cuda.synchronize()
            ts = []
            for _ in range(reps):
                e0.record()
                fn()
                e1.record()
                torch.cuda.synchronize()
                ts.append(e0.elapsed_time(e1) * 1e3 / rounds)
            return statistics.median(ts)

        us = timed(lambda: L.barrier_probe_launches(vp(out.data_ptr()), words, rounds, grid, stream))
        print(f"words {words}: separate launches {us:.2f} us per round", flush=True)
        for mode, name in ((0, "no fences"), (1, "per-WG release + acquire"),
                           (2, "per-XCD wbl2 + per-WG acquire"), (3, "per-WG release only")):
            def run():
                ctl.zero_()
                assert L.barrier_probe_fused(vp(out.data_ptr()), words, rounds, mode, vp(ctl.data_ptr()),
                                             vp(err.data_ptr()), grid, stream) == 0
            us = timed(run)
            print(f"words {words}: fused, {name}: {us:.2f} us per round (err {int(err.item())})", flush=True)
    xcds = ctl[32:40].cpu().tolist()
    print("workgroups per XCC:", xcds, "XCCs:", int(ctl[48].item()))


if __name__ == "__main__":
    main()
