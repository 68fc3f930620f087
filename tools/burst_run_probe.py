#!/usr/bin/env python3
"""Small bursts are latency-bound: a wave streams its run of datagrams with 4 pieces in flight, so a
run of 16 x 1500 B costs ~6 memory round trips whatever the burst size. GPU time (HIP events) of
RxBurst / TxBurst on a mixed IPv4/IPv6 ring of 1500-B frames by burst size and run length
(NETCSUM_TUNE_TILE = datagrams per wave; 0 = the library's default choice).

  python tools/burst_run_probe.py > gpurun_out/TAG_burst_run_probe.jsonl
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
    L = 1500
    nmax = 1 << 20
    pk = ring(dev, nmax, L, 0, L, 0)
    act = torch.zeros(nmax, dtype=torch.uint8, device=dev)
    netcsum.tx_burst(pk, nmax, stride=L, pkt_len=L, stream=st)
    torch.cuda.synchronize()
    for n in (64, 256, 1024, 4096, 16384, 65536, 262144, 1048576):
        for tile in (0, 1, 2, 4, 8, 16):
            netcsum.tune(netcsum.TUNE_TILE, tile if tile else -1)
            rx = events_ms(lambda: netcsum.rx_burst(pk, n, act, stride=L, pkt_len=L, stream=st), st, reps=50)
            d = netcsum.last_launch()
            tx = events_ms(lambda: netcsum.tx_burst(pk, n, stride=L, pkt_len=L, stream=st), st, reps=50)
            ok = bool((act[:n] == 0).all().item())
            print(json.dumps({"frames": n, "tile": tile, "rx_us": round(rx * 1e3, 2), "tx_us": round(tx * 1e3, 2),
                              "all_delivered": ok, "kernel": d}), flush=True)
    netcsum.tune(netcsum.TUNE_TILE, -1)


if __name__ == "__main__":
    main()
