#!/usr/bin/env python3
"""Cost of the per-call scratch lease (netcsum_abi.hip ScratchLease: an event recorded after the
launches that use a slot; a stream wait on it when the previous call's launches are pending), read
through product launch options that take the lease or not, interleaved on one box:

  C4 (1 M packed 40-9000 B + 12 B)   adaptive runs (lease: run word)   vs  VARLEN_RUN_BYTES 0 (no lease)
  Tx 1 M x 1500 B IPv4/TCP           two passes (lease: records)       vs  TX_PASSES 1 (no lease)

Round 2 measured (no lease existed then) C4 0.666-0.667 vs 0.6745-0.677 ms and Tx 0.2876-0.2882 vs
0.2957-0.2961 ms on one box; a lease cost shows as a smaller gap or a reversal.
Prints one JSON line per pass."""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for sub in ("uc-tcp-ip_amd", "oracle", "", "tools"):
    sys.path.insert(0, os.path.join(REPO, sub))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import netcsum  # noqa: E402
from bench import SEED  # noqa: E402
from bench_configs import events_ms  # noqa: E402


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
    ph = torch.zeros(nv * 12, dtype=torch.uint8, device=dev)
    off_d = torch.from_numpy(off.view(np.int64)).to(dev)
    len_d = torch.from_numpy(lens.view(np.int16)).to(dev)
    o4 = torch.empty(nv, dtype=torch.int16, device=dev)
    n, L = 1 << 20, 1500
    pk = torch.empty(n * L + 256, dtype=torch.uint8, device=dev)
    netcsum.fill(pk, n * L, SEED, 0)
    v = pk[: n * L].view(n, L)
    v[:, 0:12] = torch.tensor([0x45, 0, L >> 8, L & 0xFF, 0, 0, 0x40, 0, 64, 6, 0, 0], dtype=torch.uint8, device=dev)

    def c4():
        netcsum.batch_varlen(base, off_d, len_d, ph, 12, 12, nv, o4, 0, stream=st)

    def tx():
        netcsum.tx_finalize_ipv4(pk, n, None, stride=L, pkt_len=L, stream=st)

    for rep in range(3):
        r = {"pass": rep}
        for name, fn, key, on, off_v in (("C4", c4, netcsum.TUNE_VARLEN_RUN_BYTES, -1, 0),
                                         ("tx_v4", tx, netcsum.TUNE_TX_PASSES, 0, 1)):
            netcsum.tune(key, on)
            r[name + "_lease_ms"] = round(events_ms(fn, st, reps=40), 4)
            netcsum.tune(key, off_v)
            r[name + "_nolease_ms"] = round(events_ms(fn, st, reps=40), 4)
            netcsum.tune(key, on)
        print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
