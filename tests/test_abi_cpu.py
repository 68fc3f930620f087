"""CPU-side checks of the product C ABI (no kernel launches):

* libnetcsum_mi355x.so loads and exports every function include/netcsum_mi355x.h declares;
* the gfx950 code object is embedded (the library is a HIP fat binary for gfx950 only);
* the NET_BUF chain walk (host logic of net_util.c:1589-1687) yields exactly the byte stream of the
  numpy oracle's stream view, for random chains, every protocol type, odd pseudo-headers, the
  NULL-chain quirk and the DBG-mode errors;
* argument validation errors are returned before any device work;
* without a GPU the per-packet functions FAIL LOUDLY (NET_UTIL_ERR_MI355X_DEV) — there is no CPU
  fallback to silently produce numbers.
"""
import ctypes
import os
import random
import subprocess

import pytest

import netcsum
import oracle_np as onp
from conftest import gpu_available
from helpers import rand_bytes, rand_chain, to_np_buf


def test_library_exports_every_header_symbol():
    L = netcsum.lib()
    names = netcsum.exported_symbols_from_headers()
    assert len(names) >= 13
    for n in names:
        assert hasattr(L, n), f"{n} declared in include/netcsum_mi355x.h but not exported"
    assert netcsum.version().endswith("gfx950")


def test_library_carries_gfx950_code_object():
    """The .hip_fatbin section embeds an amdgcn code object whose target id is gfx950."""
    blob = open(netcsum.LIB_PATH, "rb").read()
    assert b"amdgcn-amd-amdhsa--gfx950" in blob
    for other in (b"--gfx942", b"--gfx90a", b"--gfx1100"):
        assert other not in blob


def _stream_bytes(spans):
    return b"".join(ctypes.string_at(p, ln) for p, ln in spans)


@pytest.mark.parametrize("seed", range(6))
def test_chain_to_spans_matches_stream_view(seed):
    rng = random.Random(seed)
    for _ in range(120):
        nbuf = rng.randint(1, 5)
        chain = rand_chain(rng, rng.randint(0, 2000), nbuf)
        plen = rng.choice([0, 1, 11, 12, 40])
        pseudo = rand_bytes(rng, plen) if rng.random() < 0.8 else None
        ch = netcsum.Chain(chain)
        ph = netcsum.HostBytes(pseudo, rng.randint(0, 7)) if pseudo is not None else None
        spans, err = netcsum.chain_to_spans(ch.ptr, ph.ptr if ph else None, plen if ph else 0)
        want, werr = onp.chain_stream([to_np_buf(b) for b in chain], pseudo)
        assert err == werr == 200
        assert _stream_bytes(spans) == want


def test_chain_to_spans_quirks_and_errors():
    ph = netcsum.HostBytes(b"\x01\x02\x03")
    spans, err = netcsum.chain_to_spans(None, ph.ptr, 3)          # NULL chain: odd octet dropped
    assert err == 200 and _stream_bytes(spans) == b"\x01\x02"
    bad = netcsum.Chain([{"data": b"ab", "proto": 71}, {"data": b"cd", "proto": 62}])
    assert netcsum.chain_to_spans(bad.ptr, None, 0)[1] == 211
    assert netcsum.chain_to_spans(None, None, 0, dbg=True)[1] == 23
    empty = netcsum.Chain([{"data": b"", "proto": 70}])
    assert netcsum.chain_to_spans(empty.ptr, None, 0, dbg=True)[1] == 210
    assert netcsum.chain_to_spans(empty.ptr, None, 0, dbg=False) == ([], 200)
    ix = netcsum.Chain([{"data": b"abcd", "proto": 71, "transport_ix": 0xFFFF, "data_len": 0}])
    assert netcsum.chain_to_spans(ix.ptr, None, 0, dbg=True)[1] == 622
    many = netcsum.Chain([{"data": b"ab", "proto": 71}] * 10)
    spans, err = netcsum.chain_to_spans(many.ptr, None, 0, max_spans=4)      # caller's array too small:
    assert err == netcsum.NET_UTIL_ERR_BUF_TOO_SMALL and len(spans) == 4      # first 4 + the count needed
    spans, err = netcsum.chain_to_spans(many.ptr, None, 0)                   # auto-sized: all 10
    assert err == 200 and [ln for _, ln in spans] == [2] * 10


@pytest.mark.parametrize("nbuf", [63, 64, 65, 200, 1000])
def test_chain_to_spans_long_chains_no_cap(nbuf):
    """net_util.c:1611-1687 walks chains of any length (e.g. a 64 KiB datagram reassembled from
    576-B-MTU fragments, net_ipv4.c:6523, is ~120 buffers): the walk has no span cap."""
    rng = random.Random(nbuf)
    chain = []
    for i in range(nbuf):
        ln = 0 if i % 17 == 5 else rng.randint(1, 97)                # odd splits, empty middles
        chain.append({"data": rand_bytes(rng, ln), "proto": 70 if i == 0 else 71, "offset": rng.randint(0, 3)})
    pseudo = rand_bytes(rng, 11)
    ch = netcsum.Chain(chain)
    ph = netcsum.HostBytes(pseudo, 1)
    spans, err = netcsum.chain_to_spans(ch.ptr, ph.ptr, 11)
    want, werr = onp.chain_stream([to_np_buf(b) for b in chain], pseudo)
    assert err == werr == 200
    assert _stream_bytes(spans) == want
    n = ctypes.c_uint32(7)
    assert netcsum.lib().NetUtil_MI355X_ChainToSpans(ch.ptr, ph.ptr, 11, None, 0, ctypes.byref(n), 0) == 200
    assert n.value == len(spans)


def test_batch_argument_validation_before_device_work():
    L = netcsum.lib()
    # HDR ops take no pseudo-header
    assert L.NetUtil_MI355X_ChkSumBatchStrided(1, 20, 20, 8, 12, 12, 4, 16, netcsum.OP_HDR_CALC, None) == 219
    assert L.NetUtil_MI355X_ChkSumBatchStrided(1, 20, 20, None, 0, 0, 4, 16, 7, None) == 219
    assert L.NetUtil_MI355X_ChkSumBatchStrided(None, 20, 20, None, 0, 0, 4, 16, 0, None) == 23
    assert L.NetUtil_MI355X_ChkSumBatchStrided(None, 20, 20, None, 0, 0, 0, None, 0, None) == 200   # n=0
    assert L.NetUtil_MI355X_ChkSumBatchVarLen(8, None, 8, None, 0, 0, 4, 16, 0, None) == 23
    assert L.NetUtil_MI355X_Tune(netcsum.TUNE_GROUP_LANES, 3) == 219
    assert L.NetUtil_MI355X_Tune(netcsum.TUNE_BLOCK_THREADS, 512) == 219
    assert L.NetUtil_MI355X_Tune(99, 1) == 219
    assert L.NetUtil_MI355X_Tune(31, 0) == 219                                 # no such key
    assert L.NetUtil_MI355X_Tune(netcsum.TUNE_CHAIN_GRID, 17) == 219           # -1 .. 16
    assert L.NetUtil_MI355X_Tune(netcsum.TUNE_CHAIN_GRID, -1) == 200
    assert L.NetUtil_MI355X_Tune(netcsum.TUNE_CHAIN_COMBINE, 32) == 219        # -1, 16 or 64
    assert L.NetUtil_MI355X_Tune(netcsum.TUNE_CHAIN_COMBINE, -1) == 200
    assert L.NetUtil_MI355X_Tune(netcsum.TUNE_STORE_GATHER, 2) == 219          # -1, 0 or 1
    assert L.NetUtil_MI355X_Tune(netcsum.TUNE_LIVE_COMPACT, 2) == 219          # -1, 0 or 1
    assert L.NetUtil_MI355X_Tune(netcsum.TUNE_PLAN_AHEAD, 2) == 219            # -1, 0 or 1
    assert L.NetUtil_MI355X_Tune(netcsum.TUNE_PLAN_AHEAD, -1) == 200
    assert L.NetUtil_MI355X_PlanBind(7) == 200 and L.NetUtil_MI355X_PlanBind(0) == 200
    assert L.NetUtil_MI355X_Tune(netcsum.TUNE_BURST_ZERO_COPY, 4) == 219       # 0..3
    assert L.NetUtil_MI355X_Tune(netcsum.TUNE_BURST_SERVER_IDLE_US, 0) == 219  # 1..10^6
    assert L.NetUtil_MI355X_Tune(netcsum.TUNE_BURST_SERVER_IDLE_US, 500) == 200
    assert L.NetUtil_MI355X_Tune(netcsum.TUNE_BURST_SERVER_LIFE_US, 0) == 219  # 1..10^6
    assert L.NetUtil_MI355X_Tune(netcsum.TUNE_BURST_SERVER_LIFE_US, 1000) == 200
    assert L.NetUtil_MI355X_Tune(netcsum.TUNE_FAULT_INJECT, 2) == 219          # 0 or 1 (test only)
    assert L.NetUtil_MI355X_Tune(netcsum.TUNE_FAULT_INJECT, 0) == 200
    assert L.NetUtil_MI355X_Tune(netcsum.TUNE_PKT_BOUND, 5) == 219             # -1..4
    assert L.NetUtil_MI355X_Tune(netcsum.TUNE_PKT_BOUND, -1) == 200
    assert L.NetUtil_MI355X_Tune(netcsum.TUNE_VARLEN_RUN_BYTES, -2) == 219     # -1 .. 2^20
    assert L.NetUtil_MI355X_Tune(netcsum.TUNE_HDR_BURST, 2) == 219             # 0 or 1
    assert L.NetUtil_MI355X_Tune(netcsum.TUNE_CRC_KERNEL, 4) == 219            # 0..3
    assert L.NetUtil_MI355X_Tune(netcsum.TUNE_CRC_LANES, 3) == 219             # 0, 1, 2, 4, 8, 16
    assert L.NetUtil_MI355X_Tune(netcsum.TUNE_CRC_WIDE, 3) == 219              # 0, 1 or 2
    assert L.NetUtil_MI355X_Tune(netcsum.TUNE_CRC_NT, -1) == 219               # 0 or 1
    assert L.NetUtil_MI355X_Tune(netcsum.TUNE_TX_FLUSH, 5) == 219              # -1..4
    assert L.NetUtil_MI355X_Tune(netcsum.TUNE_STREAM_XCD, 4097) == 219       # -1 .. 4096
    assert L.NetUtil_MI355X_Tune(netcsum.TUNE_STREAM_XCD, -2) == 219
    assert L.NetUtil_MI355X_Tune(netcsum.TUNE_STREAM_TOUCH, 2) == 219          # -1, 0 or 1
    assert L.NetUtil_MI355X_Tune(netcsum.TUNE_STREAM_WAVES, 2) == 219          # 3..8 or 0
    assert L.NetUtil_MI355X_Tune(netcsum.TUNE_TX_PASSES, 3) == 219
    assert L.NetUtil_MI355X_Fill(3, 10, 0, 0, 0, None) == 219                   # not 8-B aligned
    assert L.NetUtil_MI355X_ReadStream(16, 17, 8, None) == 219                # not a multiple of 16
    # strided packet batches: a stride whose 32-bit store offsets would wrap is refused (G = 8 for
    # 1500-B packets -> 7 strides + 64 KiB must stay below 2^32), checked before any device work
    big = (1 << 32) // 7
    assert L.NetUtil_MI355X_TxFinalizeIPv4(16, None, None, big, 1500, 4, None, 1, None) in (219, 218)


@pytest.mark.skipif(gpu_available(), reason="checks the no-GPU behaviour")
def test_no_gpu_fails_loudly_without_fallback():
    hb = netcsum.HostBytes(bytes.fromhex("450000730000400040110000c0a80001c0a800c7"))
    v, err = netcsum.HdrCalc(hb.ptr, 20)
    assert (v, err) == (0, netcsum.NET_UTIL_ERR_MI355X_DEV)
    ch = netcsum.Chain([{"data": b"abcdef", "proto": 71}])
    assert netcsum.DataVerify(ch.ptr, None, 0) == (0, netcsum.NET_UTIL_ERR_MI355X_DEV)
    assert netcsum.stream_sum32([(hb.ptr, 20)])[1] == netcsum.NET_UTIL_ERR_MI355X_DEV
    assert netcsum.SumDataCalcAlign_32(hb.ptr, 20) == 0         # no error channel: 0 + stderr


def test_header_is_plain_c():
    """include/*.h compile as C89-ish C11 with no HIP/torch types (the drop-in boundary)."""
    inc = os.path.join(netcsum.REPO, "include")
    src = '#include "netcsum_mi355x.h"\n#include "netcsum_netbuf.h"\nint main(void){return 0;}\n'
    r = subprocess.run(["gcc", "-std=c11", "-Wall", "-Werror", "-pedantic", "-I", inc, "-x", "c", "-",
                        "-fsyntax-only"], input=src, capture_output=True, text=True)
    assert r.returncode == 0, r.stderr


def test_binding_rejects_undersized_buffers_before_launch():
    """Host-side shape checks: an undersized tensor never reaches a kernel."""
    import numpy as np
    seg = np.zeros(1000, np.uint8)
    out = np.zeros(10, np.uint16)
    with pytest.raises(ValueError):
        netcsum.batch_strided(seg, 100, 100, None, 0, 0, 11, out, 0, stream=0)      # 1100 B > 1000
    with pytest.raises(ValueError):
        netcsum.batch_strided(seg, 100, 100, None, 0, 0, 10, out[:9], 0, stream=0)  # out too small
    ph = np.zeros(100, np.uint8)
    with pytest.raises(ValueError):
        netcsum.batch_strided(seg, 100, 100, ph, 12, 12, 10, out, 0, stream=0)      # 120 B pseudo > 100
    with pytest.raises(ValueError):
        netcsum.batch_varlen(seg, np.zeros(9, np.uint64), np.zeros(10, np.uint16), None, 0, 0, 10, out, 0, stream=0)
    # host-memory varlen: pseudo-headers and the segments' extent are checked too (the C side copies them)
    off, ln = np.arange(10, dtype=np.uint64) * 90, np.full(10, 90, np.uint16)
    with pytest.raises(ValueError):
        netcsum.batch_varlen_host(seg, off, ln, ph, 12, 12, 10, out)                 # 120 B pseudo > 100
    with pytest.raises(ValueError):
        netcsum.batch_varlen_host(seg[:899], off, ln, None, 0, 0, 10, out)           # extent 900 B > 899


def test_host_memory_forms_check_arguments_before_device_work():
    """(2e) host-memory forms: empty batches succeed, NULL pointers and bad configurations are
    rejected before any device work (so on this CPU-only host too)."""
    L = netcsum.lib()
    E_NULL, E_ARG, OK = netcsum.NET_ERR_FAULT_NULL_PTR, netcsum.NET_UTIL_ERR_MI355X_INVALID_ARG, netcsum.NET_UTIL_ERR_NONE
    assert L.NetUtil_MI355X_ChkSumBatchVarLenHost(None, None, None, None, 0, 0, 0, None, 0, 4) == OK
    assert L.NetUtil_MI355X_ChkSumBatchVarLenHost(None, None, None, None, 0, 0, 5, None, 0, 4) == E_NULL
    assert L.NetUtil_MI355X_ChkSumBatchVarLenHost(8, 8, 8, None, 0, 0, 5, 8, 7, 4) == E_ARG       # op
    assert L.NetUtil_MI355X_RxValidateIPHost(8, None, None, 64, 64, 0, None, 4) == OK
    assert L.NetUtil_MI355X_RxValidateIPHost(8, None, None, 64, 64, 3, None, 4) == E_NULL        # flags
    assert L.NetUtil_MI355X_RxValidateIPHost(None, None, None, 64, 64, 3, 8, 4) == E_NULL
    assert L.NetUtil_MI355X_RxValidateIPHost(8, 8, None, 64, 64, 3, 8, 4) == E_NULL              # off w/o len
    assert L.NetUtil_MI355X_TxFinalizeIPHost(None, None, None, 64, 64, 3, None, 1, 4) == E_NULL
    assert L.NetUtil_MI355X_RxBurstHost(8, None, None, 64, 64, 3, 0, None, None, 4) == E_NULL    # actions
    assert L.NetUtil_MI355X_RxBurstHost(8, None, None, 64, 64, 3, 4, 8, None, 4) == E_ARG        # rx_cfg
    assert L.NetUtil_MI355X_TxBurstHost(None, None, None, 64, 64, 3, None, 4) == E_NULL

