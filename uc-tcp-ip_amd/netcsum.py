"""ctypes binding of libnetcsum_mi355x.so (the C ABI in include/netcsum_mi355x.h).

Mirrors the reference's interface for the checksum path (µC/TCP-IP V3.06.01 Source/net_util.h:
422-438): the four per-packet functions keep their names, argument meaning and error behaviour
(`(value, NET_ERR)` pairs here instead of the `p_err` out-parameter), and a NET_BUF ctypes mirror
(`NetBuf`, layout of include/netcsum_netbuf.h / Source/net_buf.h:394-598 under the template
configuration) lets Python build packet chains exactly as the stack would hand them over.

The batch ABI is exposed for device-resident data: pass torch tensors (their data_ptr is used) or
raw integer device addresses, plus a HIP stream handle (defaults to torch's current stream).

There is no Python or CPU fallback: if the shared library is missing, import of the GPU entry
points raises; if the device is missing, calls return NET_UTIL_ERR_MI355X_DEV (218).
"""
from __future__ import annotations

import ctypes
import os
import re

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
# NETCSUM_LIB: an experiment build of the same library (tools/ variant sweeps); default = the in-tree build
LIB_PATH = os.environ.get("NETCSUM_LIB") or os.path.join(HERE, "libnetcsum_mi355x.so")
HEADER_PATHS = [os.path.join(REPO, "include", "netcsum_mi355x.h")]

# NET_ERR values (Source/net_err.h:73,122-126,193 + the MI355X additions in netcsum_types.h)
NET_ERR_FAULT_NULL_PTR = 23
NET_UTIL_ERR_NONE = 200
NET_UTIL_ERR_NULL_SIZE = 210
NET_UTIL_ERR_INVALID_PROTOCOL = 211
NET_UTIL_ERR_BUF_TOO_SMALL = 212
NET_UTIL_ERR_MI355X_DEV = 218
NET_UTIL_ERR_MI355X_INVALID_ARG = 219
NET_BUF_ERR_INVALID_IX = 622

# NET_PROTOCOL_TYPE (Source/net_type.h:184-235)
NET_PROTOCOL_TYPE_IP_V6_EXT_NONE = 48
NET_PROTOCOL_TYPE_ICMP_V4 = 60
NET_PROTOCOL_TYPE_ICMP_V6 = 61
NET_PROTOCOL_TYPE_IGMP = 62
NET_PROTOCOL_TYPE_UDP_V4 = 70
NET_PROTOCOL_TYPE_TCP_V4 = 71
NET_PROTOCOL_TYPE_UDP_V6 = 72
NET_PROTOCOL_TYPE_TCP_V6 = 73

DEF_OK, DEF_FAIL = 1, 0

OP_DATA_CALC, OP_DATA_VERIFY, OP_HDR_CALC, OP_HDR_VERIFY = 0, 1, 2, 3
PKT_IP_OK, PKT_L4_OK, PKT_L4_CHECKED, PKT_UDP_NO_CSUM = 0x01, 0x02, 0x04, 0x08
PKT_MALFORMED, PKT_FRAGMENT, PKT_L4_MALFORMED = 0x10, 0x20, 0x40
PKT_EXT_HDR = 0x80
# Rx burst actions / config (include/netcsum_mi355x.h (2b''): the reference's checksum-offload seam)
RX_DELIVER, RX_DROP_IPV4_CHK_SUM, RX_DROP_TCP_CHK_SUM, RX_DROP_UDP_CHK_SUM = 0, 1, 2, 3
RX_DROP_UDP_NO_CHK_SUM, RX_DROP_ICMPV4_CHK_SUM, RX_DROP_IGMP_CHK_SUM, RX_DROP_ICMPV6_CHK_SUM = 4, 5, 6, 7
RX_DELIVER_L4_UNVERIFIED, RX_NBR_ACTIONS = 8, 9
RXCFG_UDP_DISCARD_NO_CHK_SUM = 0x1
TUNE_GRID_BLOCKS, TUNE_GROUP_LANES, TUNE_NT_LOADS, TUNE_BLOCK_THREADS = 1, 2, 3, 4
TUNE_KERNEL, TUNE_CHUNKS, TUNE_PROBE, TUNE_GRID_MULT, TUNE_TILE = 5, 6, 7, 8, 9
TUNE_TX_PASSES = 10
TUNE_STREAM_WAVES = 11
TUNE_STREAM_TOUCH = 12
TUNE_STREAM_XCD = 13
TUNE_TX_FLUSH = 14
TUNE_CRC_KERNEL = 15
TUNE_CRC_NT = 16
TUNE_CRC_LANES = 17
TUNE_CRC_WIDE = 18
TUNE_HDR_BURST = 19
TUNE_VARLEN_RUN_BYTES = 20
TUNE_PKT_BOUND = 21
TUNE_BURST_ZERO_COPY = 22
TUNE_BURST_SERVER_IDLE_US = 23
TUNE_BURST_SERVER_LIFE_US = 24
TUNE_FAULT_INJECT = 25          # test only: the next offset/length packet batch skips its deferred pass and fails
TUNE_PLAN_AHEAD = 26            # first batch on a layout: sample it first and run in its plan (-1 auto, 0, 1)
TUNE_LIVE_COMPACT = 27          # live-sector streams: live sectors compacted (-1 default / 1) or live pieces (0)
TUNE_STORE_GATHER = 28          # dense segment stream: a block's results stored as whole lines (-1 / 1) or per wave (0)
TUNE_CHAIN_GRID = 29            # chain pass 1: tiles of 64 pieces per block (-1 / 0) or k x resident blocks, equal shares
TUNE_CHAIN_COMBINE = 30         # chain combine pass of the one-record form: 16 or 64 lanes per chain (-1 default)


# --------------------------------------------------------------------------- NET_BUF mirror
class NetBufHdr(ctypes.Structure):
    _fields_ = [
        ("_rsvd_000", ctypes.c_uint8 * 6),
        ("Flags", ctypes.c_uint16),
        ("_rsvd_008", ctypes.c_uint8 * 64),
        ("NextBufPtr", ctypes.c_void_p),
        ("_rsvd_080", ctypes.c_uint8 * 24),
        ("ProtocolHdrType", ctypes.c_int32),
        ("_rsvd_108", ctypes.c_uint8 * 38),
        ("ICMP_MsgIx", ctypes.c_uint16),
        ("ICMP_MsgLen", ctypes.c_uint16),
        ("ICMP_HdrLen", ctypes.c_uint16),
        ("IGMP_MsgIx", ctypes.c_uint16),
        ("IGMP_MsgLen", ctypes.c_uint16),
        ("TransportHdrIx", ctypes.c_uint16),
        ("TransportHdrLen", ctypes.c_uint16),
        ("TransportTotLen", ctypes.c_uint16),
        ("TransportDataLen", ctypes.c_uint16),
        ("DataIx", ctypes.c_uint16),
        ("DataLen", ctypes.c_uint16),
        ("TotLen", ctypes.c_uint16),
        ("_rsvd_170", ctypes.c_uint8 * 134),
    ]


class NetBuf(ctypes.Structure):
    _fields_ = [("Hdr", NetBufHdr), ("DataPtr", ctypes.c_void_p)]


assert ctypes.sizeof(NetBufHdr) == 304 and ctypes.sizeof(NetBuf) == 312
assert NetBufHdr.NextBufPtr.offset == 72 and NetBufHdr.ProtocolHdrType.offset == 104
assert NetBufHdr.ICMP_MsgIx.offset == 146 and NetBufHdr.ICMP_HdrLen.offset == 150
assert NetBufHdr.TransportHdrIx.offset == 156 and NetBufHdr.TransportHdrLen.offset == 158
assert NetBufHdr.DataLen.offset == 166 and NetBufHdr.TotLen.offset == 168


class Span(ctypes.Structure):
    _fields_ = [("p", ctypes.c_void_p), ("len", ctypes.c_uint32), ("rsvd", ctypes.c_uint32)]


class Chain:
    """A NET_BUF chain over host byte arrays (kept alive by this object).

    Each buffer: dict(data=bytes, proto=…, transport_ix=…, transport_hdr_len=…, data_len=…,
    icmp_ix=…, icmp_hdr_len=…, tot_len=…) — the fields net_util.c:1613-1640 reads.
    `offset` places the data area at an odd/unaligned address inside a larger allocation.
    """

    def __init__(self, bufs, offset: int = 0):
        self._keep = []
        self.bufs = (NetBuf * max(1, len(bufs)))()
        for i, b in enumerate(bufs):
            data = bytes(b.get("data", b""))
            off = int(b.get("offset", offset))
            arr = (ctypes.c_uint8 * (len(data) + off + 16))()
            ctypes.memmove(ctypes.addressof(arr) + off, data, len(data))
            self._keep.append(arr)
            nb = self.bufs[i]
            nb.DataPtr = ctypes.addressof(arr) + off
            h = nb.Hdr
            h.ProtocolHdrType = int(b.get("proto", NET_PROTOCOL_TYPE_TCP_V4))
            h.TransportHdrIx = int(b.get("transport_ix", 0))
            h.TransportHdrLen = int(b.get("transport_hdr_len", 0))
            h.DataLen = int(b.get("data_len", len(data) - int(b.get("transport_ix", 0))))
            h.ICMP_MsgIx = int(b.get("icmp_ix", 0))
            h.ICMP_HdrLen = int(b.get("icmp_hdr_len", 0))
            h.TotLen = int(b.get("tot_len", 0))
            h.NextBufPtr = None
        for i in range(len(bufs) - 1):
            self.bufs[i].Hdr.NextBufPtr = ctypes.addressof(self.bufs[i + 1])
        self.n = len(bufs)

    @property
    def ptr(self):
        return ctypes.addressof(self.bufs[0]) if self.n else None


class HostBytes:
    """Bytes placed at a chosen misalignment in a ctypes buffer (for pseudo-headers / headers)."""

    def __init__(self, data: bytes, offset: int = 0):
        data = bytes(data)
        self.arr = (ctypes.c_uint8 * (len(data) + offset + 16))()
        ctypes.memmove(ctypes.addressof(self.arr) + offset, data, len(data))
        self.ptr = ctypes.addressof(self.arr) + offset
        self.len = len(data)


# --------------------------------------------------------------------------- library loading
_lib = None


def exported_symbols_from_headers() -> list[str]:
    """Every function name declared in include/netcsum_mi355x.h."""
    names = []
    for p in HEADER_PATHS:
        txt = open(p).read()
        txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
        names += re.findall(r"\b(NetUtil_\w+)\s*\(", txt)
    return sorted(set(names))


def lib() -> ctypes.CDLL:
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise RuntimeError(f"{LIB_PATH} is missing — build it with `make -C {HERE}` (no fallback exists)")
    L = ctypes.CDLL(LIB_PATH)
    vp, u16, u32, u64, i32 = ctypes.c_void_p, ctypes.c_uint16, ctypes.c_uint32, ctypes.c_uint64, ctypes.c_int
    perr = ctypes.POINTER(ctypes.c_int32)
    L.NetUtil_16BitOnesCplChkSumHdrCalc.argtypes = [vp, u16, perr]
    L.NetUtil_16BitOnesCplChkSumHdrCalc.restype = u16
    L.NetUtil_16BitOnesCplChkSumHdrVerify.argtypes = [vp, u16, perr]
    L.NetUtil_16BitOnesCplChkSumHdrVerify.restype = ctypes.c_uint8
    L.NetUtil_16BitOnesCplChkSumDataCalc.argtypes = [vp, vp, u16, perr]
    L.NetUtil_16BitOnesCplChkSumDataCalc.restype = u16
    L.NetUtil_16BitOnesCplChkSumDataVerify.argtypes = [vp, vp, u16, perr]
    L.NetUtil_16BitOnesCplChkSumDataVerify.restype = ctypes.c_uint8
    L.NetUtil_MI355X_ChkSumBatchStrided.argtypes = [vp, u64, u16, vp, u32, u16, u32, vp, i32, vp]
    L.NetUtil_MI355X_ChkSumBatchStrided.restype = i32
    L.NetUtil_MI355X_ChkSumBatchVarLen.argtypes = [vp, vp, vp, vp, u32, u16, u32, vp, i32, vp]
    L.NetUtil_MI355X_ChkSumBatchVarLen.restype = i32
    L.NetUtil_MI355X_ChkSumBatchChains.argtypes = [vp, vp, vp, vp, vp, u32, u16, u32, vp, i32, vp]
    L.NetUtil_MI355X_ChkSumBatchChains.restype = i32
    L.NetUtil_MI355X_ChkSumBatchStridedHost.argtypes = [vp, u64, u16, vp, u32, u16, u32, vp, i32, u32]
    L.NetUtil_MI355X_ChkSumBatchStridedHost.restype = i32
    L.NetUtil_16BitSumDataCalcAlign_32.argtypes = [vp, u32]
    L.NetUtil_16BitSumDataCalcAlign_32.restype = u32
    L.NetUtil_MI355X_StreamSum32.argtypes = [ctypes.POINTER(Span), u32, ctypes.POINTER(ctypes.c_uint32)]
    L.NetUtil_MI355X_StreamSum32.restype = i32
    L.NetUtil_MI355X_ShardVarLen.argtypes = [vp, u32, u16, u32, vp]
    L.NetUtil_MI355X_ShardVarLen.restype = i32
    L.NetUtil_MI355X_ThreadRelease.argtypes = []
    L.NetUtil_MI355X_ThreadRelease.restype = i32
    L.NetUtil_MI355X_ChainToSpans.argtypes = [vp, vp, u16, ctypes.POINTER(Span), u32,
                                              ctypes.POINTER(ctypes.c_uint32), i32]
    L.NetUtil_MI355X_ChainToSpans.restype = i32
    L.NetUtil_MI355X_RxValidateIPv4.argtypes = [vp, vp, vp, u64, u16, u32, vp, vp]
    L.NetUtil_MI355X_RxValidateIPv4.restype = i32
    L.NetUtil_MI355X_TxFinalizeIPv4.argtypes = [vp, vp, vp, u64, u16, u32, vp, i32, vp]
    L.NetUtil_MI355X_TxFinalizeIPv4.restype = i32
    L.NetUtil_MI355X_RxValidateIPv6.argtypes = [vp, vp, vp, u64, u16, u32, vp, vp]
    L.NetUtil_MI355X_RxValidateIPv6.restype = i32
    L.NetUtil_MI355X_TxFinalizeIPv6.argtypes = [vp, vp, vp, u64, u16, u32, vp, i32, vp]
    L.NetUtil_MI355X_TxFinalizeIPv6.restype = i32
    L.NetUtil_MI355X_RxValidateIP.argtypes = [vp, vp, vp, u64, u16, u32, vp, vp]
    L.NetUtil_MI355X_RxValidateIP.restype = i32
    L.NetUtil_MI355X_TxFinalizeIP.argtypes = [vp, vp, vp, u64, u16, u32, vp, i32, vp]
    L.NetUtil_MI355X_TxFinalizeIP.restype = i32
    L.NetUtil_MI355X_RxBurst.argtypes = [vp, vp, vp, u64, u16, u32, u32, vp, vp, vp]
    L.NetUtil_MI355X_RxBurst.restype = i32
    L.NetUtil_MI355X_TxBurst.argtypes = [vp, vp, vp, u64, u16, u32, vp, vp]
    L.NetUtil_MI355X_TxBurst.restype = i32
    L.NetUtil_MI355X_RxAction.argtypes = [ctypes.c_uint8, ctypes.c_uint8, i32, u32]
    L.NetUtil_MI355X_RxAction.restype = ctypes.c_uint8
    L.NetUtil_MI355X_RxBurstTally.argtypes = [vp, u32, vp]
    L.NetUtil_MI355X_RxBurstTally.restype = i32
    L.NetUtil_MI355X_ChkSumBatchVarLenHost.argtypes = [vp, vp, vp, vp, u32, u16, u32, vp, i32, u32]
    L.NetUtil_MI355X_ChkSumBatchVarLenHost.restype = i32
    L.NetUtil_MI355X_RxValidateIPHost.argtypes = [vp, vp, vp, u64, u16, u32, vp, u32]
    L.NetUtil_MI355X_RxValidateIPHost.restype = i32
    L.NetUtil_MI355X_TxFinalizeIPHost.argtypes = [vp, vp, vp, u64, u16, u32, vp, i32, u32]
    L.NetUtil_MI355X_TxFinalizeIPHost.restype = i32
    L.NetUtil_MI355X_RxBurstHost.argtypes = [vp, vp, vp, u64, u16, u32, u32, vp, vp, u32]
    L.NetUtil_MI355X_RxBurstHost.restype = i32
    L.NetUtil_MI355X_TxBurstHost.argtypes = [vp, vp, vp, u64, u16, u32, vp, u32]
    L.NetUtil_MI355X_TxBurstHost.restype = i32
    L.NetUtil_32BitCRC_Calc.argtypes = [vp, u32, perr]
    L.NetUtil_32BitCRC_Calc.restype = u32
    L.NetUtil_32BitCRC_CalcCpl.argtypes = [vp, u32, perr]
    L.NetUtil_32BitCRC_CalcCpl.restype = u32
    L.NetUtil_32BitReflect.argtypes = [u32]
    L.NetUtil_32BitReflect.restype = u32
    L.NetUtil_MI355X_CRC32BatchStrided.argtypes = [vp, u64, u32, u32, vp, i32, vp]
    L.NetUtil_MI355X_CRC32BatchStrided.restype = i32
    L.NetUtil_MI355X_CRC32BatchVarLen.argtypes = [vp, vp, vp, u32, vp, i32, vp]
    L.NetUtil_MI355X_CRC32BatchVarLen.restype = i32
    L.NetUtil_MI355X_CRC32Host.argtypes = [vp, u32, ctypes.POINTER(ctypes.c_uint32)]
    L.NetUtil_MI355X_CRC32Host.restype = i32
    L.NetUtil_MI355X_Fill.argtypes = [vp, u64, u64, u64, i32, vp]
    L.NetUtil_MI355X_Fill.restype = i32
    L.NetUtil_MI355X_ReadStream.argtypes = [vp, u64, vp, vp]
    L.NetUtil_MI355X_ReadStream.restype = i32
    L.NetUtil_MI355X_Tune.argtypes = [i32, i32]
    L.NetUtil_MI355X_Tune.restype = i32
    L.NetUtil_MI355X_PlanBind.argtypes = [u32]
    L.NetUtil_MI355X_PlanBind.restype = i32
    L.NetUtil_MI355X_LastLaunch.argtypes = []
    L.NetUtil_MI355X_LastLaunch.restype = ctypes.c_char_p
    L.NetUtil_MI355X_Version.argtypes = []
    L.NetUtil_MI355X_Version.restype = ctypes.c_char_p
    _lib = L
    return L


def _p(x):
    """Pointer from a torch tensor, numpy array, ctypes object, int or None."""
    if x is None:
        return None
    if isinstance(x, int):
        return x
    if hasattr(x, "data_ptr"):
        return x.data_ptr()
    if hasattr(x, "ctypes"):
        return x.ctypes.data
    return ctypes.addressof(x)


def _stream(stream):
    if stream is None:
        import torch
        return torch.cuda.current_stream().cuda_stream
    if hasattr(stream, "cuda_stream"):
        return stream.cuda_stream
    return int(stream)


def _nbytes(x):
    if hasattr(x, "numel") and hasattr(x, "element_size"):
        return int(x.numel()) * int(x.element_size())
    if hasattr(x, "nbytes"):
        return int(x.nbytes)
    return None


def _require(x, need, what):
    """Host-side bounds check before any launch (a device fault can take the GPU down)."""
    have = _nbytes(x)
    if have is not None and have < need:
        raise ValueError(f"{what}: buffer holds {have} B but the launch would touch {need} B")


def _check(err, what):
    if err != NET_UTIL_ERR_NONE:
        raise RuntimeError(f"{what} returned NET_ERR {err}")


# --------------------------------------------------------------------- reference interface
def HdrCalc(phdr, hdr_size):
    err = ctypes.c_int32(0)
    v = lib().NetUtil_16BitOnesCplChkSumHdrCalc(_p(phdr), hdr_size, ctypes.byref(err))
    return int(v), int(err.value)


def HdrVerify(phdr, hdr_size):
    err = ctypes.c_int32(0)
    v = lib().NetUtil_16BitOnesCplChkSumHdrVerify(_p(phdr), hdr_size, ctypes.byref(err))
    return int(v), int(err.value)


def DataCalc(pdata_buf, ppseudo_hdr, pseudo_hdr_size):
    err = ctypes.c_int32(0)
    v = lib().NetUtil_16BitOnesCplChkSumDataCalc(_p(pdata_buf), _p(ppseudo_hdr), pseudo_hdr_size,
                                                 ctypes.byref(err))
    return int(v), int(err.value)


def DataVerify(pdata_buf, ppseudo_hdr, pseudo_hdr_size):
    err = ctypes.c_int32(0)
    v = lib().NetUtil_16BitOnesCplChkSumDataVerify(_p(pdata_buf), _p(ppseudo_hdr), pseudo_hdr_size,
                                                   ctypes.byref(err))
    return int(v), int(err.value)


def SumDataCalcAlign_32(pdata_32, size):
    """NetUtil_16BitSumDataCalcAlign_32 (net_util.h:486-490): unfolded network-order word sum."""
    return int(lib().NetUtil_16BitSumDataCalcAlign_32(_p(pdata_32), size))


def chain_to_spans(pdata_buf, ppseudo_hdr, pseudo_hdr_size, dbg=False, max_spans=None):
    """Spans of the chain's checksummed stream. max_spans=None sizes the array by a count-only
    walk first (chains of any length); a fixed max_spans returns BUF_TOO_SMALL past it, with the
    first max_spans spans and n = the count needed."""
    n = ctypes.c_uint32(0)
    if max_spans is None:
        err = lib().NetUtil_MI355X_ChainToSpans(_p(pdata_buf), _p(ppseudo_hdr), pseudo_hdr_size, None, 0,
                                                ctypes.byref(n), int(dbg))
        if err != NET_UTIL_ERR_NONE:
            return [], int(err)
        max_spans = n.value
    spans = (Span * max(1, max_spans))()
    err = lib().NetUtil_MI355X_ChainToSpans(_p(pdata_buf), _p(ppseudo_hdr), pseudo_hdr_size, spans,
                                            max_spans, ctypes.byref(n), int(dbg))
    out = [(spans[i].p, spans[i].len) for i in range(min(n.value, max_spans))]
    return out, int(err)


def shard_varlen(seg_len, pseudo_len: int, world: int):
    """Byte-balanced contiguous ranks of a varlen batch (NetUtil_MI355X_ShardVarLen): returns the
    world + 1 boundaries, rank r owning segments [first[r], first[r+1])."""
    import numpy as np
    lens = np.ascontiguousarray(seg_len, dtype=np.uint16)
    first = np.zeros(world + 1, np.uint32)
    err = lib().NetUtil_MI355X_ShardVarLen(lens.ctypes.data if lens.size else None, lens.size, pseudo_len,
                                            world, first.ctypes.data)
    if err != NET_UTIL_ERR_NONE:
        raise ValueError(f"NetUtil_MI355X_ShardVarLen: NET_ERR {err}")
    return first


def thread_release():
    """Free the calling thread's per-device drop-in contexts (also done at thread exit)."""
    return int(lib().NetUtil_MI355X_ThreadRelease())


def stream_sum32(spans):
    arr = (Span * max(1, len(spans)))()
    for i, (p, ln) in enumerate(spans):
        arr[i].p = p
        arr[i].len = ln
    s = ctypes.c_uint32(0)
    err = lib().NetUtil_MI355X_StreamSum32(arr, len(spans), ctypes.byref(s))
    return int(s.value), int(err)


# --------------------------------------------------------------------------- CRC-32 (net_util.c:485-636)
def CRC32Calc(p_data, data_len, cpl=False):
    """The drop-in NetUtil_32BitCRC_Calc / _CalcCpl on a host pointer -> (crc, err)."""
    err = ctypes.c_int32()
    f = lib().NetUtil_32BitCRC_CalcCpl if cpl else lib().NetUtil_32BitCRC_Calc
    v = f(p_data, data_len, ctypes.byref(err))
    return int(v), int(err.value)


def Reflect32(val):
    return int(lib().NetUtil_32BitReflect(val))


def crc32_strided(base, stride, length, n, out, cpl=False, stream=None, check=True):
    if n:
        _require(base, (n - 1) * stride + length, "segments")
        _require(out, 4 * n, "out")
    err = lib().NetUtil_MI355X_CRC32BatchStrided(_p(base), stride, length, n, _p(out), int(cpl), _stream(stream))
    if check:
        _check(err, "NetUtil_MI355X_CRC32BatchStrided")
    return err


def crc32_varlen(base, off, lens, n, out, cpl=False, stream=None, check=True):
    if n:
        _require(off, 8 * n, "offsets")
        _require(lens, 4 * n, "lengths")
        _require(out, 4 * n, "out")
    err = lib().NetUtil_MI355X_CRC32BatchVarLen(_p(base), _p(off), _p(lens), n, _p(out), int(cpl), _stream(stream))
    if check:
        _check(err, "NetUtil_MI355X_CRC32BatchVarLen")
    return err


# --------------------------------------------------------------------------- batch interface
def batch_strided(seg, seg_stride, seg_len, pseudo, pseudo_stride, pseudo_len, n_seg, out,
                  op=OP_DATA_CALC, stream=None, check=True):
    if n_seg:
        _require(seg, (n_seg - 1) * seg_stride + seg_len, "segments")
        if pseudo is not None and pseudo_len:
            _require(pseudo, (n_seg - 1) * pseudo_stride + pseudo_len, "pseudo-headers")
        _require(out, n_seg * (2 if op in (OP_DATA_CALC, OP_HDR_CALC) else 1), "out")
    err = lib().NetUtil_MI355X_ChkSumBatchStrided(_p(seg), seg_stride, seg_len, _p(pseudo), pseudo_stride,
                                                  pseudo_len, n_seg, _p(out), op, _stream(stream))
    if check:
        _check(err, "NetUtil_MI355X_ChkSumBatchStrided")
    return err


def batch_varlen(base, seg_off, seg_len, pseudo, pseudo_stride, pseudo_len, n_seg, out,
                 op=OP_DATA_CALC, stream=None, check=True):
    if n_seg:
        _require(seg_off, 8 * n_seg, "segment offsets")
        _require(seg_len, 2 * n_seg, "segment lengths")
        if pseudo is not None and pseudo_len:
            _require(pseudo, (n_seg - 1) * pseudo_stride + pseudo_len, "pseudo-headers")
        _require(out, n_seg * (2 if op in (OP_DATA_CALC, OP_HDR_CALC) else 1), "out")
    err = lib().NetUtil_MI355X_ChkSumBatchVarLen(_p(base), _p(seg_off), _p(seg_len), _p(pseudo), pseudo_stride,
                                                 pseudo_len, n_seg, _p(out), op, _stream(stream))
    if check:
        _check(err, "NetUtil_MI355X_ChkSumBatchVarLen")
    return err


def batch_strided_host(seg, seg_stride, seg_len, pseudo, pseudo_stride, pseudo_len, n_seg, out,
                       op=OP_DATA_CALC, n_chunks=0, check=True):
    if n_seg:
        _require(seg, (n_seg - 1) * seg_stride + seg_len, "segments")
        if pseudo is not None and pseudo_len:
            _require(pseudo, (n_seg - 1) * pseudo_stride + pseudo_len, "pseudo-headers")
        _require(out, n_seg * (2 if op in (OP_DATA_CALC, OP_HDR_CALC) else 1), "out")
    err = lib().NetUtil_MI355X_ChkSumBatchStridedHost(_p(seg), seg_stride, seg_len, _p(pseudo), pseudo_stride,
                                                      pseudo_len, n_seg, _p(out), op, n_chunks)
    if check:
        _check(err, "NetUtil_MI355X_ChkSumBatchStridedHost")
    return err


def batch_chains(base, piece_off, piece_len, chain_first, pseudo, pseudo_stride, pseudo_len, n_chains, out,
                 op=OP_DATA_CALC, stream=None, check=True, n_pieces=None):
    """Checksum n_chains NET_BUF chains (pieces [chain_first[i], chain_first[i+1]) after pseudo-header i).
    n_pieces (= chain_first[n_chains], if the caller knows it) bounds-checks the piece arrays."""
    if n_chains:
        _require(chain_first, 4 * (n_chains + 1), "chain index")
        if n_pieces is not None and n_pieces:
            _require(piece_off, 8 * n_pieces, "piece offsets")
            _require(piece_len, 2 * n_pieces, "piece lengths")
        if pseudo is not None and pseudo_len:
            _require(pseudo, (n_chains - 1) * pseudo_stride + pseudo_len, "pseudo-headers")
        _require(out, n_chains * (2 if op == OP_DATA_CALC else 1), "out")
    err = lib().NetUtil_MI355X_ChkSumBatchChains(_p(base), _p(piece_off), _p(piece_len), _p(chain_first), _p(pseudo),
                                                 pseudo_stride, pseudo_len, n_chains, _p(out), op, _stream(stream))
    if check:
        _check(err, "NetUtil_MI355X_ChkSumBatchChains")
    return err


def _pkt_bounds(base, off, lens, stride, pkt_len, n, flags):
    if not n:
        return
    if off is not None:
        _require(off, 8 * n, "packet offsets")
        _require(lens, 2 * n, "packet lengths")
    else:
        _require(base, (n - 1) * stride + pkt_len, "packets")
    if flags is not None:
        _require(flags, n, "flags")


def rx_validate_ipv4(base, n, flags, off=None, lens=None, stride=0, pkt_len=0, stream=None, check=True):
    _pkt_bounds(base, off, lens, stride, pkt_len, n, flags)
    err = lib().NetUtil_MI355X_RxValidateIPv4(_p(base), _p(off), _p(lens), stride, pkt_len, n, _p(flags),
                                              _stream(stream))
    if check:
        _check(err, "NetUtil_MI355X_RxValidateIPv4")
    return err


def tx_finalize_ipv4(base, n, flags=None, off=None, lens=None, stride=0, pkt_len=0, udp_tx_csum=True,
                     stream=None, check=True):
    _pkt_bounds(base, off, lens, stride, pkt_len, n, flags)
    err = lib().NetUtil_MI355X_TxFinalizeIPv4(_p(base), _p(off), _p(lens), stride, pkt_len, n, _p(flags),
                                              int(bool(udp_tx_csum)), _stream(stream))
    if check:
        _check(err, "NetUtil_MI355X_TxFinalizeIPv4")
    return err


def rx_validate_ipv6(base, n, flags, off=None, lens=None, stride=0, pkt_len=0, stream=None, check=True):
    _pkt_bounds(base, off, lens, stride, pkt_len, n, flags)
    err = lib().NetUtil_MI355X_RxValidateIPv6(_p(base), _p(off), _p(lens), stride, pkt_len, n, _p(flags),
                                              _stream(stream))
    if check:
        _check(err, "NetUtil_MI355X_RxValidateIPv6")
    return err


def tx_finalize_ipv6(base, n, flags=None, off=None, lens=None, stride=0, pkt_len=0, udp_tx_csum=True,
                     stream=None, check=True):
    _pkt_bounds(base, off, lens, stride, pkt_len, n, flags)
    err = lib().NetUtil_MI355X_TxFinalizeIPv6(_p(base), _p(off), _p(lens), stride, pkt_len, n, _p(flags),
                                              int(bool(udp_tx_csum)), _stream(stream))
    if check:
        _check(err, "NetUtil_MI355X_TxFinalizeIPv6")
    return err


def rx_validate_ip(base, n, flags, off=None, lens=None, stride=0, pkt_len=0, stream=None, check=True):
    """Mixed IPv4 / IPv6 batch: per packet by the version nibble."""
    _pkt_bounds(base, off, lens, stride, pkt_len, n, flags)
    err = lib().NetUtil_MI355X_RxValidateIP(_p(base), _p(off), _p(lens), stride, pkt_len, n, _p(flags),
                                            _stream(stream))
    if check:
        _check(err, "NetUtil_MI355X_RxValidateIP")
    return err


def tx_finalize_ip(base, n, flags=None, off=None, lens=None, stride=0, pkt_len=0, udp_tx_csum=True,
                   stream=None, check=True):
    _pkt_bounds(base, off, lens, stride, pkt_len, n, flags)
    err = lib().NetUtil_MI355X_TxFinalizeIP(_p(base), _p(off), _p(lens), stride, pkt_len, n, _p(flags),
                                            int(bool(udp_tx_csum)), _stream(stream))
    if check:
        _check(err, "NetUtil_MI355X_TxFinalizeIP")
    return err


def rx_burst(base, n, action, flags=None, off=None, lens=None, stride=0, pkt_len=0, rx_cfg=0, stream=None,
             check=True):
    """NetUtil_MI355X_RxBurst: per-frame NETCSUM_RX_* actions of a mixed IPv4 / IPv6 burst."""
    _pkt_bounds(base, off, lens, stride, pkt_len, n, flags)
    if n:
        _require(action, n, "actions")
    err = lib().NetUtil_MI355X_RxBurst(_p(base), _p(off), _p(lens), stride, pkt_len, n, rx_cfg, _p(action),
                                       _p(flags), _stream(stream))
    if check:
        _check(err, "NetUtil_MI355X_RxBurst")
    return err


def tx_burst(base, n, flags=None, off=None, lens=None, stride=0, pkt_len=0, stream=None, check=True):
    """NetUtil_MI355X_TxBurst: fill in the checksum fields the stack left to the offload, in place."""
    _pkt_bounds(base, off, lens, stride, pkt_len, n, flags)
    err = lib().NetUtil_MI355X_TxBurst(_p(base), _p(off), _p(lens), stride, pkt_len, n, _p(flags), _stream(stream))
    if check:
        _check(err, "NetUtil_MI355X_TxBurst")
    return err


def rx_action(flags, proto, ipv6, rx_cfg=0):
    """NetUtil_MI355X_RxAction (host logic): the burst action of one verdict."""
    return int(lib().NetUtil_MI355X_RxAction(flags, proto, int(bool(ipv6)), rx_cfg))


def rx_burst_tally(actions):
    """NetUtil_MI355X_RxBurstTally over a host uint8 array -> list of RX_NBR_ACTIONS counts."""
    import numpy as np
    a = np.ascontiguousarray(actions, dtype=np.uint8)
    ctr = np.zeros(RX_NBR_ACTIONS, np.uint32)
    _check(lib().NetUtil_MI355X_RxBurstTally(a.ctypes.data if a.size else None, a.size, ctr.ctypes.data),
           "NetUtil_MI355X_RxBurstTally")
    return [int(x) for x in ctr]


# ------------------------------------------------------------------ host-memory forms ((2e))
def batch_varlen_host(base, seg_off, seg_len, pseudo, pseudo_stride, pseudo_len, n_seg, out, op=OP_DATA_CALC,
                      n_chunks=0, check=True):
    if n_seg:
        _require(seg_off, 8 * n_seg, "segment offsets")
        _require(seg_len, 2 * n_seg, "segment lengths")
        if pseudo is not None and pseudo_len:
            _require(pseudo, (n_seg - 1) * pseudo_stride + pseudo_len, "pseudo-headers")
        _require(out, n_seg * (2 if op in (OP_DATA_CALC, OP_HDR_CALC) else 1), "out")
        # host arrays: the segments' extent is readable here (the C side copies [min off, max off+len))
        import numpy as _np
        if isinstance(seg_off, _np.ndarray) and isinstance(seg_len, _np.ndarray) and _nbytes(base) is not None:
            o = seg_off[:n_seg].view(_np.uint64)
            ln = _np.asarray(seg_len[:n_seg]).view(_np.uint16).astype(_np.uint64)
            _require(base, int((o + ln).max()), "segments")
    err = lib().NetUtil_MI355X_ChkSumBatchVarLenHost(_p(base), _p(seg_off), _p(seg_len), _p(pseudo), pseudo_stride,
                                                     pseudo_len, n_seg, _p(out), op, n_chunks)
    if check:
        _check(err, "NetUtil_MI355X_ChkSumBatchVarLenHost")
    return err


def rx_validate_ip_host(base, n, flags, off=None, lens=None, stride=0, pkt_len=0, n_chunks=0, check=True):
    _pkt_bounds(base, off, lens, stride, pkt_len, n, flags)
    err = lib().NetUtil_MI355X_RxValidateIPHost(_p(base), _p(off), _p(lens), stride, pkt_len, n, _p(flags), n_chunks)
    if check:
        _check(err, "NetUtil_MI355X_RxValidateIPHost")
    return err


def tx_finalize_ip_host(base, n, flags=None, off=None, lens=None, stride=0, pkt_len=0, udp_tx_csum=True, n_chunks=0,
                        check=True):
    _pkt_bounds(base, off, lens, stride, pkt_len, n, flags)
    err = lib().NetUtil_MI355X_TxFinalizeIPHost(_p(base), _p(off), _p(lens), stride, pkt_len, n, _p(flags),
                                                int(bool(udp_tx_csum)), n_chunks)
    if check:
        _check(err, "NetUtil_MI355X_TxFinalizeIPHost")
    return err


def rx_burst_host(base, n, action, flags=None, off=None, lens=None, stride=0, pkt_len=0, rx_cfg=0, n_chunks=0,
                  check=True):
    _pkt_bounds(base, off, lens, stride, pkt_len, n, flags)
    if n:
        _require(action, n, "actions")
    err = lib().NetUtil_MI355X_RxBurstHost(_p(base), _p(off), _p(lens), stride, pkt_len, n, rx_cfg, _p(action),
                                           _p(flags), n_chunks)
    if check:
        _check(err, "NetUtil_MI355X_RxBurstHost")
    return err


def tx_burst_host(base, n, flags=None, off=None, lens=None, stride=0, pkt_len=0, n_chunks=0, check=True):
    _pkt_bounds(base, off, lens, stride, pkt_len, n, flags)
    err = lib().NetUtil_MI355X_TxBurstHost(_p(base), _p(off), _p(lens), stride, pkt_len, n, _p(flags), n_chunks)
    if check:
        _check(err, "NetUtil_MI355X_TxBurstHost")
    return err


def fill(buf, n_bytes, seed, pattern=0, stream=None, first_byte=0):
    _require(buf, n_bytes, "fill buffer")
    _check(lib().NetUtil_MI355X_Fill(_p(buf), n_bytes, first_byte, seed, pattern, _stream(stream)),
           "NetUtil_MI355X_Fill")


def read_stream(buf, n_bytes, sink, stream=None):
    _require(buf, n_bytes, "read-stream buffer")
    _require(sink, 8, "sink")
    _check(lib().NetUtil_MI355X_ReadStream(_p(buf), n_bytes, _p(sink), _stream(stream)),
           "NetUtil_MI355X_ReadStream")


def tune(key, value):
    _check(lib().NetUtil_MI355X_Tune(key, value), "NetUtil_MI355X_Tune")


def plan_bind(plan_id):
    """NetUtil_MI355X_PlanBind: this thread's later planned batches key their plans on plan_id too."""
    _check(lib().NetUtil_MI355X_PlanBind(plan_id), "NetUtil_MI355X_PlanBind")


def last_launch() -> str:
    return lib().NetUtil_MI355X_LastLaunch().decode()


def version() -> str:
    return lib().NetUtil_MI355X_Version().decode()
