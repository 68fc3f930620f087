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


def test_dropin_short_crc_runs_on_the_host():
    """Per-call CRCs of up to 4096 octets (the drivers' 6-octet multicast hashes) are the reference's
    register update in host C, no device round trip: they work without a GPU and equal the oracle,
    at every length 1..300 and at 4096; Reflect of them gives the drivers' 6-bit hash."""
    import random
    rng = random.Random(8)
    for n in list(range(1, 301)) + [1500, 4096]:
        m = rng.randbytes(n)
        buf = (ctypes.c_uint8 * n).from_buffer_copy(m)
        for cpl in (False, True):
            assert netcsum.CRC32Calc(ctypes.addressof(buf), n, cpl) == oracle.crc32_calc(m, cpl), (n, cpl)
    mac = (ctypes.c_uint8 * 6).from_buffer_copy(bytes([0x01, 0x00, 0x5E, 0x7F, 0x00, 0x01]))
    crc, err = netcsum.CRC32Calc(ctypes.addressof(mac), 6, True)
    assert err == netcsum.NET_UTIL_ERR_NONE
    assert netcsum.Reflect32(crc) >> 26 == oracle.reflect32(oracle.crc32_calc(bytes(mac), True)[0]) >> 26
