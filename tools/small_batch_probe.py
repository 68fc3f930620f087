#!/usr/bin/env python3
"""Small dense segment batches (C2's shape, 1500-B segments + 12-B pseudo-headers) by batch size: GPU
time of NetUtil_MI355X_ChkSumBatchStrided with the library's run choice (runs halved until the batch
spans >= 2048 waves) against C2's fixed runs of 16 (NETCSUM_TUNE_TILE 16).

  python tools/small_batch_probe.py > gpurun_out/TAG_small_batch_probe.jsonl
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
    L, nmax = 1500, 1 << 20
    seg = torch.empty(nmax * L + 256, dtype=torch.uint8, device=dev)
    netcsum.fill(seg, nmax * L, SEED, 0)
    ph = torch.zeros(nmax * 12, dtype=torch.uint8, device=dev)
    out = torch.empty(nmax, dtype=torch.int16, device=dev)
    for n in (16, 64, 256, 1024, 4096, 16384, 65536, 1048576):
        r = {"segments": n}
        for tag, tile in (("auto", -1), ("runs16", 16)):
            netcsum.tune(netcsum.TUNE_TILE, tile)
            r[tag + "_us"] = round(events_ms(lambda: netcsum.batch_strided(seg, L, L, ph, 12, 12, n, out,
                                                                           netcsum.OP_DATA_CALC, stream=st), st) * 1e3, 2)
            r["kernel_" + tag] = netcsum.last_launch()
        netcsum.tune(netcsum.TUNE_TILE, -1)
        print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
