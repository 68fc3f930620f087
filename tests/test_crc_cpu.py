"""CRC-32 of net_util.c:485-636 on the CPU side: the oracle restatement pinned to the published
CRC-32 check value ("123456789" -> 0xCBF43926, the IEEE 802.3 / zlib CRC, i.e. CalcCpl; Calc is its
complement 0x340BC6D9) and to zlib's independent implementation, the drop-in's reflect (host C) and
its argument checks (NET_ERR_CFG_ARG_CHK_EXT_EN), which return before any device work."""
import ctypes
import random
import zlib

import netcsum
import oracle


def test_oracle_crc32_known_answer_and_zlib():
    assert oracle.crc32_calc(b"123456789", cpl=True) == (0xCBF43926, 200)
    assert oracle.crc32_calc(b"123456789") == (0x340BC6D9, 200)
    rng = random.Random(5)
    for n in list(range(1, 70)) + [255, 256, 257, 1500, 4096, 9000]:
        m = bytes(rng.getrandbits(8) for _ in range(n))
        assert oracle.crc32_calc(m, cpl=True) == (zlib.crc32(m), 200), n
        assert oracle.crc32_calc(m) == (zlib.crc32(m) ^ 0xFFFFFFFF, 200), n


def test_oracle_crc32_argument_checks():
    assert oracle.crc32_calc(None) == (0, 23)                     # net_util.c:499-503
    assert oracle.crc32_calc(b"") == (0, 210)                     # :504-508
    assert oracle.crc32_calc(None, cpl=True) == (0, 23)


def test_dropin_reflect_matches_reference_loop():
    rng = random.Random(7)
    for v in [0, 1, 0x80000000, 0xFFFFFFFF, 0x12345678] + [rng.getrandbits(32) for _ in range(2000)]:
        assert netcsum.Reflect32(v) == oracle.reflect32(v), hex(v)


def test_dropin_crc_argument_checks_before_device_work():
    """NULL and zero length are answered by the host C (no GPU needed, none touched)."""
    assert netcsum.CRC32Calc(None, 6) == (0, netcsum.NET_ERR_FAULT_NULL_PTR)
    assert netcsum.CRC32Calc(None, 6, cpl=True) == (0, netcsum.NET_ERR_FAULT_NULL_PTR)
    buf = (ctypes.c_uint8 * 6)()
    assert netcsum.CRC32Calc(ctypes.addressof(buf), 0) == (0, netcsum.NET_UTIL_ERR_NULL_SIZE)
    assert netcsum.CRC32Calc(ctypes.addressof(buf), 0, cpl=True) == (0, netcsum.NET_UTIL_ERR_NULL_SIZE)


def test_crc_batch_rejects_null_before_device_work():
    L = netcsum.lib()
    assert L.NetUtil_MI355X_CRC32BatchStrided(None, 6, 6, 0, None, 0, None) == netcsum.NET_UTIL_ERR_NONE   # n = 0
    assert L.NetUtil_MI355X_CRC32BatchStrided(None, 6, 6, 4, 16, 0, None) == netcsum.NET_ERR_FAULT_NULL_PTR
    assert L.NetUtil_MI355X_CRC32BatchVarLen(8, None, 8, 4, 16, 0, None) == netcsum.NET_ERR_FAULT_NULL_PTR
