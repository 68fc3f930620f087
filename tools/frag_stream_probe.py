#!/usr/bin/env python3
"""The chain row's fragments (737 280 x 1480 B) read by the other kernel forms, to separate the access
pattern from the layout: the chain kernel and the varlen kernel at buffer pitches 1480 (contiguous),
1520 and 2048 (the chain batch in its default form and in the wave-per-chain form, TUNE_KERNEL 1),
the varlen batch also in the lane-group pipe form (TUNE_KERNEL 2), and the strided segment kernels (C2's form: runs of whole 1-KiB pieces, the gaps
read and skipped) at the same pitches; payload GB/s, two interleaved passes.

  python tools/frag_stream_probe.py > gpurun_out/TAG_frag_stream_probe.jsonl

profiles/r3s_frag_stream_probe.jsonl, by "build": r4f the product library; r4g a two-pass chain form
(flat per-piece even/odd sums in piece order, then a combine pass per chain; the chain columns are
that form and, with TUNE_KERNEL 1, the wave-per-chain kernel); r4h / r4i the same with the even/odd
sums taken as byte + half-word sums (v_sad_u8 + v_sad_u16, half the VALU ops); r4j the wave-per-chain
kernel with its descriptors batch-loaded into VGPRs (64 per vector load, read by v_readlane) instead
of scalar loads a step ahead. None of those was faster (0.195-0.200 ms throughout); none was kept.
r4k adds the varlen lane-group pipe forced to 16 lanes x 6 chunks (0.165 ms at pitch 2048, tiles of 64
segments; 0.173 grid-stride). r4l-r4n: the two-pass form rebuilt on that geometry (pass 1 in tiles
of 64 consecutive pieces, pass 2 a 16-lane group per chain): 0.191-0.197 ms, rocprof 177-180 us +
5.3 us (profiles/r3s_r4m/r4n_frag_rocprof_kernel_stats.csv) against 197 us for the wave-per-chain
kernel — the product form since r4n. r4o: pass 1 without the byte sum (timing only, wrong
results): 178 us, so the VALU of the even/odd split is not what separates it from the segment
kernel's 169 us.
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
    base = torch.empty(npc * 2048 + 256, dtype=torch.uint8, device=dev)
    netcsum.fill(base, base.numel() - 256, SEED, 0)
    payload = npc * flen
    for rep in range(2):
        for P in (1480, 1520, 2048):
            offs = (np.arange(npc, dtype=np.uint64) * P + ix).astype(np.uint64)
            off_d = torch.from_numpy(offs.view(np.int64)).to(dev)
            r = {"pass": rep, "pitch": P}
            r["chain_ms"] = events_ms(lambda: netcsum.batch_chains(base, off_d, len_d, first_d, ph, 12, 12, nc, oc, 0,
                                                                   stream=st, n_pieces=npc), st)
            r["kernel_chain"] = netcsum.last_launch()
            netcsum.tune(netcsum.TUNE_KERNEL, 1)
            r["chain_wave_ms"] = events_ms(lambda: netcsum.batch_chains(base, off_d, len_d, first_d, ph, 12, 12, nc, oc,
                                                                        0, stream=st, n_pieces=npc), st)
            r["kernel_chain_wave"] = netcsum.last_launch()
            netcsum.tune(netcsum.TUNE_KERNEL, 0)
            r["varlen_ms"] = events_ms(lambda: netcsum.batch_varlen(base, off_d, len_d, None, 0, 0, npc, os_,
                                                                    netcsum.OP_DATA_CALC, stream=st), st)
            r["kernel_varlen"] = netcsum.last_launch()
            netcsum.tune(netcsum.TUNE_KERNEL, 2)
            r["varlen_pipe_ms"] = events_ms(lambda: netcsum.batch_varlen(base, off_d, len_d, None, 0, 0, npc, os_,
                                                                         netcsum.OP_DATA_CALC, stream=st), st)
            r["kernel_varlen_pipe"] = netcsum.last_launch()
            netcsum.tune(netcsum.TUNE_GROUP_LANES, 16)
            netcsum.tune(netcsum.TUNE_CHUNKS, 6)
            r["varlen_pipe16_ms"] = events_ms(lambda: netcsum.batch_varlen(base, off_d, len_d, None, 0, 0, npc, os_,
                                                                           netcsum.OP_DATA_CALC, stream=st), st)
            r["kernel_varlen_pipe16"] = netcsum.last_launch()
            netcsum.tune(netcsum.TUNE_TILE, 0)
            r["varlen_pipe16_t0_ms"] = events_ms(lambda: netcsum.batch_varlen(base, off_d, len_d, None, 0, 0, npc, os_,
                                                                              netcsum.OP_DATA_CALC, stream=st), st)
            r["kernel_varlen_pipe16_t0"] = netcsum.last_launch()
            r["strided_t0_ms"] = events_ms(lambda: netcsum.batch_strided(base[ix:], P, flen, None, 0, 0, npc, os_,
                                                                         netcsum.OP_DATA_CALC, stream=st), st)
            r["kernel_strided_t0"] = netcsum.last_launch()
            netcsum.tune(netcsum.TUNE_TILE, -1)
            netcsum.tune(netcsum.TUNE_GROUP_LANES, 0)
            netcsum.tune(netcsum.TUNE_CHUNKS, 0)
            netcsum.tune(netcsum.TUNE_KERNEL, 0)
            r["strided_ms"] = events_ms(lambda: netcsum.batch_strided(base[ix:], P, flen, None, 0, 0, npc, os_,
                                                                      netcsum.OP_DATA_CALC, stream=st), st)
            r["kernel_strided"] = netcsum.last_launch()
            for k in ("chain", "chain_wave", "varlen", "varlen_pipe", "varlen_pipe16", "varlen_pipe16_t0", "strided",
                      "strided_t0"):
                r[k + "_ms"] = round(r[k + "_ms"], 4)
                r[k + "_GBps_payload"] = round(payload / r[k + "_ms"] / 1e6, 1)
            print(json.dumps(r), flush=True)
            del off_d


if __name__ == "__main__":
    main()
