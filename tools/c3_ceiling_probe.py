#!/usr/bin/env python3
"""Read-rate ceiling at C3's size: the 16 M x 20-B header batch (335.5 MB) against the read-stream
probe over the same bytes, and the probe over C2's 1.57 GB for comparison, two interleaved passes.
A 57-us launch pays its fill and drain on a smaller base than C2's 218 us.

  python tools/c3_ceiling_probe.py > gpurun_out/TAG_c3_ceiling.jsonl
"""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for sub in ("uc-tcp-ip_amd", "oracle", "", "tools"):
    sys.path.insert(0, os.path.join(REPO, sub))
import torch  # noqa: E402

import netcsum  # noqa: E402
from bench import SEED  # noqa: E402
from bench_configs import events_ms  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    st = torch.cuda.current_stream(dev)
    n3, n2 = 1 << 24, 1 << 20
    big = torch.empty(n2 * 1500 + 256, dtype=torch.uint8, device=dev)
    netcsum.fill(big, n2 * 1500, SEED, 0)
    out = torch.empty(n3, dtype=torch.int16, device=dev)
    sink = torch.empty(4096, dtype=torch.int32, device=dev)
    for rep in range(2):
        hdr = events_ms(lambda: netcsum.batch_strided(big, 20, 20, None, 0, 0, n3, out, netcsum.OP_HDR_CALC,
                                                      stream=st), st)
        k_hdr = netcsum.last_launch()
        for probe in (1, 2):
            netcsum.tune(netcsum.TUNE_PROBE, probe)
            r3 = events_ms(lambda: netcsum.read_stream(big, n3 * 20, sink, stream=st), st)
            r2 = events_ms(lambda: netcsum.read_stream(big, n2 * 1500, sink, stream=st), st)
            print(json.dumps({"pass": rep, "probe": probe, "c3_hdr_ms": round(hdr, 4),
                              "c3_read_probe_ms": round(r3, 4), "c2_read_probe_ms": round(r2, 4),
                              "c3_read_probe_GBps": round(n3 * 20 / r3 / 1e6, 1),
                              "c2_read_probe_GBps": round(n2 * 1500 / r2 / 1e6, 1),
                              "c3_hdr_GBps_algorithmic": round(n3 * 22 / hdr / 1e6, 1),
                              "kernel_hdr": k_hdr}), flush=True)
        netcsum.tune(netcsum.TUNE_PROBE, 1)


if __name__ == "__main__":
    main()
