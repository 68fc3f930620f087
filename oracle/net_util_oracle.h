/*
 * ORACLE — TEST INFRASTRUCTURE ONLY. Never linked into, loaded by or called from the product
 * library (uc-tcp-ip_amd/libnetcsum_mi355x.so). Only tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg may use it, and only as the checker / CPU baseline.
 *
 * CPU restatement of the µC/TCP-IP V3.06.01 Internet-checksum path (Source/net_util.c),
 * written from the reference's algorithm, not copied from it. Each function cites the
 * reference lines it restates.
 *
 * PARITY STATUS: "parity unpinned by the reference's own artefacts". The reference ships no
 * tests, fixtures or golden vectors, and its net_util.c cannot be built in this image
 * without writing stand-ins for the un-vendored Micrium uC-CPU / uC-LIB / KAL headers, which this
 * project does not do. The oracle is pinned instead by
 *   - the two published external known-answer tests (RFC 1071 §3 worked example; the classic
 *     IPv4 header 4500 0073 … → b861), tests/test_oracle_kat.py;
 *   - an independent second restatement written from RFC 1071 + SURVEY Appendix B in numpy
 *     (oracle/oracle_np.py), cross-checked on thousands of random headers, segments and
 *     NET_BUF chains, tests/test_oracle_cross.py.
 *
 * Byte-order: NET_UTIL_HOST_TO_NET_16 / NET_UTIL_NET_TO_HOST_16 (net_util.h:102,105) map to
 * uC-LIB MEM_VAL_HOST_TO_BIG_16 / MEM_VAL_BIG_TO_HOST_16 (uC-LIB >= V1.38.00, net.h:372-374;
 * not vendored). On a little-endian CPU those are a 16-bit byte swap — restated as ORC_SWAP16.
 */
#ifndef NET_UTIL_ORACLE_H
#define NET_UTIL_ORACLE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Reference public functions (net_util.c:159, :245, :344, :428). `dbg_chk` != 0 enables the
 * NET_ERR_CFG_ARG_CHK_DBG_EN argument checks (default DISABLED, Cfg/Template/net_cfg.h:184).
 * pdata_buf points at a NET_BUF laid out as include/netcsum_netbuf.h. */
uint16_t Oracle_HdrCalc   (const void *phdr, uint16_t hdr_size, uint32_t *p_err, int dbg_chk);
uint8_t  Oracle_HdrVerify (const void *phdr, uint16_t hdr_size, uint32_t *p_err, int dbg_chk);
uint16_t Oracle_DataCalc  (const void *pdata_buf, const void *ppseudo_hdr, uint16_t pseudo_hdr_size,
                           uint32_t *p_err, int dbg_chk);
uint8_t  Oracle_DataVerify(const void *pdata_buf, const void *ppseudo_hdr, uint16_t pseudo_hdr_size,
                           uint32_t *p_err, int dbg_chk);

/* The internal u32 accumulator of NetUtil_16BitOnesCplSumDataCalc before the fold
 * (net_util.c:1554-1686), for checking NetUtil_MI355X_StreamSum32. Returns the NET_ERR. */
uint32_t Oracle_DataSum32 (const void *pdata_buf, const void *ppseudo_hdr, uint16_t pseudo_hdr_size,
                           uint32_t *p_sum32);

/* Batch drivers with the semantics of the batch ABI (include/netcsum_mi355x.h (2)): each segment
 * is wrapped in a one-buffer NET_BUF (TCP_V4) and run through Oracle_DataCalc/Verify, or through
 * Oracle_HdrCalc/Verify for ops 2/3 — i.e. the reference's per-packet call, once per segment.
 * op: 0 DATA_CALC (u16 out), 1 DATA_VERIFY (u8 out), 2 HDR_CALC (u16), 3 HDR_VERIFY (u8).
 * n_threads > 1 splits segments statically over OpenMP threads (0 = OpenMP default). */
void Oracle_BatchStrided(const uint8_t *seg, uint64_t seg_stride, uint16_t seg_len,
                         const uint8_t *pseudo, uint32_t pseudo_stride, uint16_t pseudo_len,
                         uint32_t n_seg, void *out, int op, int n_threads);
void Oracle_BatchVarLen (const uint8_t *base, const uint64_t *seg_off, const uint16_t *seg_len,
                         const uint8_t *pseudo, uint32_t pseudo_stride, uint16_t pseudo_len,
                         uint32_t n_seg, void *out, int op, int n_threads);

/* splitmix64-based synthetic bytes, identical to NetUtil_MI355X_Fill (pattern 0..3), for
 * regenerating any byte range on the host. */
void Oracle_BatchChains(const uint8_t *base, const uint64_t *piece_off, const uint16_t *piece_len,
                        const uint32_t *chain_first, const uint8_t *pseudo, uint32_t pseudo_stride,
                        uint16_t pseudo_len, uint32_t n_chains, void *out, int op, int n_threads);
void Oracle_Fill(uint8_t *buf, uint64_t first_byte, uint64_t n_bytes, uint64_t seed, int pattern);
void Oracle_FillParallel(uint8_t *buf, uint64_t first_byte, uint64_t n_bytes, uint64_t seed, int pattern,
                         int n_threads, uint64_t unit);

/* The stack's per-datagram Rx (tx = 0: HdrVerify + DataVerify) or Tx (tx = 1: HdrCalc + DataCalc
 * written in place) checksum sequence over a strided batch of well-formed IPv4 / IPv6 (no extension
 * header) datagrams, OpenMP static: the CPU line of the fused packet rows (net_util_oracle.c). */
void Oracle_PktBatch(uint8_t *base, uint64_t stride, uint16_t avail, uint32_t n, int tx, uint8_t *flags,
                     int n_threads);

/* Config C1 (BASELINE configs[0]) per-datagram checksum sequence of the loopback UDP echo
 * (SURVEY §3.1/§3.2), `iters` times on the same NET_BUF: Tx DataCalc(pbuf, pseudo, plen)
 * (net_udp.c:2891) -> HdrCalc(ip_hdr, 20) (net_ipv4.c:9578) -> Rx HdrVerify(ip_hdr, 20)
 * (net_ipv4.c:5247) -> DataVerify(pbuf, pseudo, plen) (net_udp.c:1934). Returns an XOR of the
 * results (so no call is elided); bench.py times it for the C1 CPU per-call figure. */
uint32_t Oracle_C1Loop(const void *pdata_buf, const void *ppseudo_hdr, uint16_t pseudo_hdr_size,
                       const void *ip_hdr, uint64_t iters);

/* CRC-32 of net_util.c:485-636 (IEEE 802.3, reflected, init 0xFFFFFFFF; Calc without and CalcCpl
 * with the final complement; NULL -> 23, zero length -> 210 with the EXT argument checks on). */
uint32_t Oracle_CRC32Calc(const uint8_t *p_data, uint32_t data_len, uint32_t *p_err);
uint32_t Oracle_CRC32CalcCpl(const uint8_t *p_data, uint32_t data_len, uint32_t *p_err);
uint32_t Oracle_Reflect32(uint32_t val);
void     Oracle_CRC32Batch(const uint8_t *base, const uint64_t *off, const uint32_t *lens, uint64_t stride,
                           uint32_t len, uint32_t n, uint32_t *out, int cpl);

/* Number of OpenMP threads the batch drivers would use with n_threads = 0. */
int  Oracle_MaxThreads(void);

#ifdef __cplusplus
}
#endif

#endif /* NET_UTIL_ORACLE_H */
