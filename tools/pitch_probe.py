#!/usr/bin/env python3
"""Does the buffer pitch of a fragmented layout set the read rate?  The chain row (16 Ki chains x 45
fragments of 1480 B, each in its own buffer at ix 42) runs at 5.5 TB/s with 2048-B buffers, against
7.2 TB/s for packed 1500-B datagrams.  This probe keeps the fragments (count, length, ix) and varies
only the buffer pitch, timing the chain kernel and the varlen segment kernel (every fragment a
segment, no pseudo-header) on the same bytes, two interleaved passes.

  python tools/pitch_probe.py > gpurun_out/TAG_pitch_probe.jsonl
"""
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

PITCHES = (1520, 1536, 1600, 1792, 2048, 2112, 2304, 3072, 4096)


def main():
    dev = torch.device("cuda", 0)
    st = torch.cuda.current_stream(dev)
    nc, per, ix, flen = 1 << 14, 45, 42, 1480
    npc = nc * per
    lens = np.full(npc, flen, np.uint16)
    first = (np.arange(nc + 1, dtype=np.uint64) * per).astype(np.uint32)
    len_d = torch.from_numpy(lens.view(np.int16)).to(dev)
    first_d = torch.from_numpy(first.view(np.int32)).to(dev)
    ph = torch.zeros(nc * 12, dtype=torch.uint8, device=dev)
    oc = torch.empty(nc, dtype=torch.int16, device=dev)
    os_ = torch.empty(npc, dtype=torch.int16, device=dev)
    base = torch.empty(npc * max(PITCHES) + 256, dtype=torch.uint8, device=dev)
    netcsum.fill(base, base.numel() - 256, SEED, 0)
    payload = npc * flen
    for rep in range(2):
        for P in PITCHES:
            offs = (np.arange(npc, dtype=np.uint64) * P + ix).astype(np.uint64)
            off_d = torch.from_numpy(offs.view(np.int64)).to(dev)
            ch = events_ms(lambda: netcsum.batch_chains(base, off_d, len_d, first_d, ph, 12, 12, nc, oc, 0,
                                                        stream=st, n_pieces=npc), st)
            k_ch = netcsum.last_launch()
            vl = events_ms(lambda: netcsum.batch_varlen(base, off_d, len_d, None, 0, 0, npc, os_,
                                                        netcsum.OP_DATA_CALC, stream=st), st)
            k_vl = netcsum.last_launch()
            print(json.dumps({"pass": rep, "pitch": P, "ix": ix, "frag_len": flen, "fragments": npc,
                              "chain_ms": round(ch, 4), "chain_GBps": round(payload / ch / 1e6, 1),
                              "varlen_ms": round(vl, 4), "varlen_GBps": round(payload / vl / 1e6, 1),
                              "kernel_chain": k_ch, "kernel_varlen": k_vl}), flush=True)
            del off_d


if __name__ == "__main__":
    main()
