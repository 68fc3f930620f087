#!/usr/bin/env python3
"""GPU-side cost of the stream primitives a per-call scratch lease could use, measured around a
product launch (the C4 varlen batch, 0.67 ms) repeated back to back on one stream:

  plain              the launches alone
  record             + an event recorded after each launch (hipEventRecord)
  record_wait        + the stream made to wait for the previous launch's event (hipStreamWaitEvent
                       on the SAME stream: redundant ordering, the cost of the barrier packet)

Wall time per launch over 200 launches after a warm-up, three interleaved passes; prints JSON lines."""
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for sub in ("uc-tcp-ip_amd", "oracle", ""):
    sys.path.insert(0, os.path.join(REPO, sub))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import netcsum  # noqa: E402
from bench import SEED  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    st = torch.cuda.current_stream(dev)
    rng = np.random.default_rng(7)
    nv = 1 << 20
    lens = rng.integers(40, 9001, size=nv).astype(np.uint16)
    off = np.zeros(nv, np.uint64)
    off[1:] = np.cumsum(lens[:-1].astype(np.uint64))
    tot = int(off[-1]) + int(lens[-1])
    base = torch.empty(tot + 256, dtype=torch.uint8, device=dev)
    netcsum.fill(base, tot, SEED, 0)
    off_d = torch.from_numpy(off.view(np.int64)).to(dev)
    len_d = torch.from_numpy(lens.view(np.int16)).to(dev)
    o4 = torch.empty(nv, dtype=torch.int16, device=dev)
    netcsum.tune(netcsum.TUNE_VARLEN_RUN_BYTES, 0)                 # runs of 8: no scratch in the call

    def launch():
        netcsum.batch_varlen(base, off_d, len_d, None, 0, 0, nv, o4, 0, stream=st)

    evs = [torch.cuda.Event() for _ in range(2)]

    def run(mode, k=200):
        for _ in range(20):
            launch()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(k):
            if mode == "record_wait" and i:
                st.wait_event(evs[(i - 1) & 1])
            launch()
            if mode in ("record", "record_wait"):
                evs[i & 1].record(st)
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / k * 1e3

    for rep in range(3):
        print(json.dumps({"pass": rep, **{m + "_ms": round(run(m), 5) for m in ("plain", "record", "record_wait")}}),
              flush=True)


if __name__ == "__main__":
    main()
