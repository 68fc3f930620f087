"""ORACLE — test infrastructure only (ctypes loader for oracle/build/liboracle_netutil.so).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this module, and
only as the checker / CPU baseline. The product library never links or calls it.

The C restatement it loads is documented in oracle/net_util_oracle.h (parity status: pinned by
external RFC 1071 / IPv4 KATs and by the independent numpy restatement oracle/oracle_np.py;
"parity unpinned" by the reference's own artefacts, which do not exist).
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "build", "liboracle_netutil.so")
_lib = None

OP_DATA_CALC, OP_DATA_VERIFY, OP_HDR_CALC, OP_HDR_VERIFY = 0, 1, 2, 3


def build() -> str:
    """Compile the C restatement with gcc (oracle/Makefile)."""
    subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return _LIB_PATH


def build_native(out_dir: str, cc: str = "gcc") -> str:
    """The same C restatement built for THIS host's CPU (-O3 -march=native): bench.py's "best CPU"
    line. Built where it runs (the GPU box's host), never shipped."""
    out = os.path.join(out_dir, "liboracle_netutil_native.so")
    subprocess.run([cc, "-O3", "-march=native", "-std=gnu11", "-fPIC", "-fopenmp", "-shared", "-o", out,
                    os.path.join(_HERE, "net_util_oracle.c")], check=True, timeout=120)
    return out


def batch_strided_with(path: str, seg: np.ndarray, seg_stride: int, seg_len: int, pseudo, pseudo_stride: int,
                       pseudo_len: int, n_seg: int, op: int = OP_DATA_CALC, n_threads: int = 1) -> np.ndarray:
    """batch_strided through another build of the restatement (build_native)."""
    L = _bind(ctypes.CDLL(path))
    out = _out_array(n_seg, op)
    L.Oracle_BatchStrided(seg.ctypes.data, seg_stride, seg_len, _ptr(pseudo), pseudo_stride, pseudo_len,
                          n_seg, out.ctypes.data, op, n_threads)
    return out


def lib() -> ctypes.CDLL:
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        _lib = _bind(ctypes.CDLL(_LIB_PATH))
    return _lib


def _bind(L: ctypes.CDLL) -> ctypes.CDLL:
    vp, u16, u32, u64, i32 = ctypes.c_void_p, ctypes.c_uint16, ctypes.c_uint32, ctypes.c_uint64, ctypes.c_int
    pu32 = ctypes.POINTER(ctypes.c_uint32)
    L.Oracle_HdrCalc.argtypes = [vp, u16, pu32, i32]
    L.Oracle_HdrCalc.restype = u16
    L.Oracle_HdrVerify.argtypes = [vp, u16, pu32, i32]
    L.Oracle_HdrVerify.restype = ctypes.c_uint8
    L.Oracle_DataCalc.argtypes = [vp, vp, u16, pu32, i32]
    L.Oracle_DataCalc.restype = u16
    L.Oracle_DataVerify.argtypes = [vp, vp, u16, pu32, i32]
    L.Oracle_DataVerify.restype = ctypes.c_uint8
    L.Oracle_DataSum32.argtypes = [vp, vp, u16, pu32]
    L.Oracle_DataSum32.restype = u32
    L.Oracle_BatchStrided.argtypes = [vp, u64, u16, vp, u32, u16, u32, vp, i32, i32]
    L.Oracle_BatchStrided.restype = None
    L.Oracle_BatchVarLen.argtypes = [vp, vp, vp, vp, u32, u16, u32, vp, i32, i32]
    L.Oracle_BatchVarLen.restype = None
    L.Oracle_BatchChains.argtypes = [vp, vp, vp, vp, vp, u32, u16, u32, vp, i32, i32]
    L.Oracle_BatchChains.restype = None
    L.Oracle_Fill.argtypes = [vp, u64, u64, u64, i32]
    L.Oracle_Fill.restype = None
    L.Oracle_FillParallel.argtypes = [vp, u64, u64, u64, i32, i32, u64]
    L.Oracle_FillParallel.restype = None
    L.Oracle_C1Loop.argtypes = [vp, vp, u16, vp, u64]
    L.Oracle_C1Loop.restype = u32
    L.Oracle_CRC32Calc.argtypes = [vp, u32, pu32]
    L.Oracle_CRC32Calc.restype = u32
    L.Oracle_CRC32CalcCpl.argtypes = [vp, u32, pu32]
    L.Oracle_CRC32CalcCpl.restype = u32
    L.Oracle_Reflect32.argtypes = [u32]
    L.Oracle_Reflect32.restype = u32
    L.Oracle_CRC32Batch.argtypes = [vp, vp, vp, u64, u32, u32, vp, i32]
    L.Oracle_CRC32Batch.restype = None
    L.Oracle_PktBatch.argtypes = [vp, u64, u16, u32, i32, vp, i32]
    L.Oracle_PktBatch.restype = None
    L.Oracle_MaxThreads.argtypes = []
    L.Oracle_MaxThreads.restype = i32
    return L


def _ptr(a):
    if a is None:
        return None
    if isinstance(a, int):
        return a
    if isinstance(a, np.ndarray):
        return a.ctypes.data
    return ctypes.cast(a, ctypes.c_void_p).value


# ----------------------------------------------------------------------------- per-packet API
def hdr_calc(ptr, size, dbg=False):
    err = ctypes.c_uint32(0)
    v = lib().Oracle_HdrCalc(_ptr(ptr), size, ctypes.byref(err), int(dbg))
    return int(v), int(err.value)


def hdr_verify(ptr, size, dbg=False):
    err = ctypes.c_uint32(0)
    v = lib().Oracle_HdrVerify(_ptr(ptr), size, ctypes.byref(err), int(dbg))
    return int(v), int(err.value)


def data_calc(pbuf, pseudo, pseudo_size, dbg=False):
    err = ctypes.c_uint32(0)
    v = lib().Oracle_DataCalc(_ptr(pbuf), _ptr(pseudo), pseudo_size, ctypes.byref(err), int(dbg))
    return int(v), int(err.value)


def data_verify(pbuf, pseudo, pseudo_size, dbg=False):
    err = ctypes.c_uint32(0)
    v = lib().Oracle_DataVerify(_ptr(pbuf), _ptr(pseudo), pseudo_size, ctypes.byref(err), int(dbg))
    return int(v), int(err.value)


def data_sum32(pbuf, pseudo, pseudo_size):
    s = ctypes.c_uint32(0)
    err = lib().Oracle_DataSum32(_ptr(pbuf), _ptr(pseudo), pseudo_size, ctypes.byref(s))
    return int(s.value), int(err)


# ----------------------------------------------------------------------------- batch drivers
def _out_array(n, op):
    return np.zeros(n, dtype=np.uint16 if op in (OP_DATA_CALC, OP_HDR_CALC) else np.uint8)


def batch_strided(seg: np.ndarray, seg_stride: int, seg_len: int, pseudo, pseudo_stride: int,
                  pseudo_len: int, n_seg: int, op: int = OP_DATA_CALC, n_threads: int = 1,
                  seg_offset: int = 0) -> np.ndarray:
    """Reference semantics of NetUtil_MI355X_ChkSumBatchStrided over host numpy buffers."""
    out = _out_array(n_seg, op)
    base = seg.ctypes.data + seg_offset
    lib().Oracle_BatchStrided(base, seg_stride, seg_len, _ptr(pseudo), pseudo_stride, pseudo_len,
                              n_seg, out.ctypes.data, op, n_threads)
    return out


def batch_varlen(base: np.ndarray, seg_off: np.ndarray, seg_len: np.ndarray, pseudo, pseudo_stride: int,
                 pseudo_len: int, op: int = OP_DATA_CALC, n_threads: int = 1) -> np.ndarray:
    seg_off = np.ascontiguousarray(seg_off, dtype=np.uint64)
    seg_len = np.ascontiguousarray(seg_len, dtype=np.uint16)
    n = int(seg_off.shape[0])
    out = _out_array(n, op)
    lib().Oracle_BatchVarLen(base.ctypes.data, seg_off.ctypes.data, seg_len.ctypes.data, _ptr(pseudo),
                             pseudo_stride, pseudo_len, n, out.ctypes.data, op, n_threads)
    return out


def batch_chains(base: np.ndarray, piece_off: np.ndarray, piece_len: np.ndarray, chain_first: np.ndarray,
                 pseudo, pseudo_stride: int, pseudo_len: int, n_chains: int, op: int = 0,
                 n_threads: int = 0) -> np.ndarray:
    """Reference per-chain DataCalc/DataVerify over NET_BUF chains built from the piece spans."""
    piece_off = np.ascontiguousarray(piece_off, np.uint64)
    piece_len = np.ascontiguousarray(piece_len, np.uint16)
    chain_first = np.ascontiguousarray(chain_first, np.uint32)
    assert len(chain_first) >= n_chains + 1 and int(chain_first[n_chains]) <= len(piece_off)
    out = _out_array(n_chains, op)
    lib().Oracle_BatchChains(base.ctypes.data, piece_off.ctypes.data, piece_len.ctypes.data, chain_first.ctypes.data,
                             _ptr(pseudo), pseudo_stride, pseudo_len, n_chains, out.ctypes.data, op, n_threads)
    return out


def fill(first_byte: int, n_bytes: int, seed: int, pattern: int = 0) -> np.ndarray:
    buf = np.empty(n_bytes, dtype=np.uint8)
    lib().Oracle_Fill(buf.ctypes.data, first_byte, n_bytes, seed, pattern)
    return buf


def fill_parallel(first_byte: int, n_bytes: int, seed: int, pattern: int = 0, n_threads: int = 0,
                  unit: int = 0) -> np.ndarray:
    """fill(), first-touched by the OpenMP workers in the static partition of `unit`-byte items."""
    buf = np.empty(n_bytes, dtype=np.uint8)
    lib().Oracle_FillParallel(buf.ctypes.data, first_byte, n_bytes, seed, pattern, n_threads, unit)
    return buf


def c1_loop(pbuf, pseudo, pseudo_size, ip_hdr, iters: int) -> int:
    """The C1 per-datagram sequence (DataCalc, HdrCalc, HdrVerify, DataVerify) `iters` times in C."""
    return int(lib().Oracle_C1Loop(_ptr(pbuf), _ptr(pseudo), pseudo_size, _ptr(ip_hdr), iters))


def max_threads() -> int:
    return int(lib().Oracle_MaxThreads())


# ---- CRC-32 (net_util.c:485-636) -----------------------------------------------------------

def crc32_calc(data, cpl: bool = False):
    """(crc, err) of NetUtil_32BitCRC_Calc / _CalcCpl over `data` (bytes, or None for NULL)."""
    err = ctypes.c_uint32()
    if data is None:
        p, n = None, 0
    else:
        buf = (ctypes.c_uint8 * max(1, len(data))).from_buffer_copy(bytes(data) or b"\0")
        p, n = ctypes.addressof(buf), len(data)
    f = lib().Oracle_CRC32CalcCpl if cpl else lib().Oracle_CRC32Calc
    return int(f(p, n, ctypes.byref(err))), int(err.value)


def reflect32(v: int) -> int:
    return int(lib().Oracle_Reflect32(v))


def crc32_batch(base: np.ndarray, n: int, cpl: bool, stride: int = 0, length: int = 0, off=None, lens=None):
    out = np.zeros(n, np.uint32)
    o = None if off is None else np.ascontiguousarray(off, np.uint64)
    ln = None if lens is None else np.ascontiguousarray(lens, np.uint32)
    lib().Oracle_CRC32Batch(base.ctypes.data, None if o is None else o.ctypes.data,
                            None if ln is None else ln.ctypes.data, stride, length, n, out.ctypes.data, int(cpl))
    return out


def pkt_batch(base: np.ndarray, stride: int, avail: int, n: int, tx: bool, n_threads: int = 1) -> np.ndarray:
    """The stack's per-datagram Rx / Tx checksum sequence over a strided batch (Oracle_PktBatch; Tx
    writes the fields into `base`): flags bit 0 IP OK, bit 1 transport OK, bit 2 transport checked."""
    flags = np.zeros(n, np.uint8)
    lib().Oracle_PktBatch(base.ctypes.data, stride, avail, n, int(bool(tx)), flags.ctypes.data, n_threads)
    return flags
