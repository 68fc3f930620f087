#!/usr/bin/env python3
"""Where a small burst's fixed cost goes: 200 back-to-back RxBurst / TxBurst calls of 256 frames on an
IPv4 ring and on a mixed IPv4/IPv6 ring, to be run under `rocprofv3 --kernel-trace` (kernel durations
and the gaps between them), with the HIP-event time per call printed beside.

  cd /tmp && rocprofv3 --kernel-trace -d $R/gpurun_out/TAG_burst_trace -o tr --output-format csv \\
      -- python3 $R/tools/burst_overhead_trace.py
"""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for sub in ("uc-tcp-ip_amd", "oracle", "", "tools"):
    sys.path.insert(0, os.path.join(REPO, sub))
import torch  # noqa: E402

import netcsum  # noqa: E402
from bench_configs import events_ms  # noqa: E402
from tx_sector_probe import ring  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    st = torch.cuda.current_stream(dev)
    n, L = 256, 1500
    for ver, tag in ((4, "v4"), (0, "mixed")):
        pk = ring(dev, n, L, 0, L, ver)
        act = torch.zeros(n, dtype=torch.uint8, device=dev)
        netcsum.tx_burst(pk, n, stride=L, pkt_len=L, stream=st)
        torch.cuda.synchronize()
        rx = events_ms(lambda: netcsum.rx_burst(pk, n, act, stride=L, pkt_len=L, stream=st), st, reps=200)
        d_rx = netcsum.last_launch()
        tx = events_ms(lambda: netcsum.tx_burst(pk, n, stride=L, pkt_len=L, stream=st), st, reps=200)
        d_tx = netcsum.last_launch()
        print(json.dumps({"ring": tag, "frames": n, "rx_us": round(rx * 1e3, 2), "tx_us": round(tx * 1e3, 2),
                          "kernel_rx": d_rx, "kernel_tx": d_tx}), flush=True)


if __name__ == "__main__":
    main()
