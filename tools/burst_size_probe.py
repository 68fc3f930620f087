#!/usr/bin/env python3
"""Burst size for the offload seam: what one RxBurst / TxBurst call costs as a
function of the number of frames, against the reference's per-frame checksum calls on one host core.

Frames: 1500-B IPv4/TCP and IPv6/TCP alternating (checksums made valid by one TxBurst). Per burst
size n:
  * device-resident RxBurst / TxBurst: the GPU time (HIP events) and the synchronous wall time of one
    call (call + hipStreamSynchronize, median of 50), i.e. what a driver thread waits;
  * host-memory RxBurstHost / TxBurstHost from pinned memory: wall time of one call (they return
    with the results in host memory);
  * CPU: the C restatement's per-datagram sequence (Oracle_PktBatch: HdrVerify + DataVerify on Rx,
    HdrCalc + DataCalc on Tx) over the same n frames on one thread.

  python tools/burst_size_probe.py > gpurun_out/TAG_burst_size_probe.jsonl
"""
import json
import os
import statistics
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for sub in ("uc-tcp-ip_amd", "oracle", "", "tools"):
    sys.path.insert(0, os.path.join(REPO, sub))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import netcsum  # noqa: E402
import oracle  # noqa: E402
from bench_configs import events_ms  # noqa: E402
from tx_sector_probe import ring  # noqa: E402

SIZES = (1, 16, 64, 256, 1024, 4096, 16384, 65536, 262144, 1048576)


def wall_us(fn, reps=50):
    for _ in range(5):
        fn()
    t = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        t.append(time.perf_counter() - t0)
    return statistics.median(t) * 1e6


def main():
    dev = torch.device("cuda", 0)
    st = torch.cuda.current_stream(dev)
    nmax, L = SIZES[-1], 1500
    pk = ring(dev, nmax, L, 0, L, 0)
    netcsum.tx_burst(pk, nmax, stride=L, pkt_len=L, stream=st)              # valid checksums
    act = torch.zeros(nmax, dtype=torch.uint8, device=dev)
    pk_h = pk[: nmax * L].cpu().pin_memory()
    act_h = torch.zeros(nmax, dtype=torch.uint8).pin_memory()
    host = pk_h.numpy()
    torch.cuda.synchronize()
    for n in SIZES:
        r = {"frames": n, "bytes": n * L}
        r["rx_gpu_us"] = round(events_ms(lambda: netcsum.rx_burst(pk, n, act, stride=L, pkt_len=L, stream=st), st) * 1e3, 2)
        r["tx_gpu_us"] = round(events_ms(lambda: netcsum.tx_burst(pk, n, stride=L, pkt_len=L, stream=st), st) * 1e3, 2)

        def rx_sync():
            netcsum.rx_burst(pk, n, act, stride=L, pkt_len=L, stream=st)
            st.synchronize()

        def tx_sync():
            netcsum.tx_burst(pk, n, stride=L, pkt_len=L, stream=st)
            st.synchronize()
        r["rx_sync_wall_us"] = round(wall_us(rx_sync), 2)
        r["tx_sync_wall_us"] = round(wall_us(tx_sync), 2)
        chunks = 1 if n < 4096 else 8
        r["rx_host_wall_us"] = round(wall_us(lambda: netcsum.rx_burst_host(pk_h, n, act_h, stride=L, pkt_len=L,
                                                                            n_chunks=chunks), reps=20), 2)
        r["tx_host_wall_us"] = round(wall_us(lambda: netcsum.tx_burst_host(pk_h, n, None, stride=L, pkt_len=L,
                                                                            n_chunks=chunks), reps=20), 2)
        reps = max(1, min(50, 20000 // n))
        r["rx_cpu_1thread_us"] = round(wall_us(lambda: oracle.pkt_batch(host, L, L, n, False, n_threads=1),
                                               reps=reps), 2)
        r["tx_cpu_1thread_us"] = round(wall_us(lambda: oracle.pkt_batch(host, L, L, n, True, n_threads=1),
                                               reps=reps), 2)
        r["rx_all_delivered"] = bool((act[:n] == 0).all().item()) and bool((act_h[:n] == 0).all().item())
        print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
