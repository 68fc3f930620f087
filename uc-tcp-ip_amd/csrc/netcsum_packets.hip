// netcsum_packets.hip — gfx950 IPv4 packet-batch kernels.
//
// RX (fused validation, one HBM pass per packet): for every received IPv4 datagram
//   ip_ok = NetUtil_16BitOnesCplChkSumHdrVerify(ip_hdr, IHL*4)               net_ipv4.c:5247
//   l4_ok = TCP : DataVerify(seg, {src,dst,0,6,  IP datagram len}, 12)        net_tcp.c:7857
//           UDP : checksum field 0 -> "no checksum", accepted                 net_udp.c:1916-1920,1971
//                 else DataVerify(dgram, {src,dst,0,17, UDP len}, 12)         net_udp.c:1934
//           ICMP: DataVerify(msg, NULL, 0)                                    net_icmpv4.c:1676
//           IGMP: HdrVerify(msg, msg len)                                     net_igmp.c:1332
//   with the pseudo-header built in registers from the IP header, instead of two passes
//   (header verify, then transport verify) over HBM.
// TX (finalize, in place): the same sums with the checksum fields treated as zero (callers zero
//   them first, net_ipv4.c:9573), then the checksums are written back:
//   IP header (offset 10)                 NetUtil_16BitOnesCplChkSumHdrCalc   net_ipv4.c:9578,9586
//   TCP (hlen+16)                         DataCalc + pseudo-header            net_tcp.c:29824,29862
//   UDP (hlen+6), 0x0000 -> 0xFFFF        DataCalc + pseudo-header            net_udp.c:2891,2929-2937
//       (or 0 when UDP Tx checksums are disabled, NET_UDP_CFG_TX_CHK_SUM_EN, net_udp.c:2935)
//   ICMP / IGMP (hlen+2)                  DataCalc / HdrCalc                  net_icmpv4.c:2204, net_igmp.c:1692
//
// Validation order follows the reference: a malformed IPv4 header (version, IHL, total length
// vs. bytes received; net_ipv4.c:5123-5254) or transport length (net_tcp.c:7808-7818,
// net_udp.c:1893-1907) means no checksum verdict for that layer. Fragments (MF or offset != 0)
// get the IP verdict only: their transport checksum covers the reassembled datagram
// (net_ipv4.c:6523), which a per-packet batch does not have.
//
// Work decomposition: the pipelined v2 structure of netcsum_kernels.hip (G >= 8 lanes per
// packet, K chunks per lane per pass, the next packet's loads in flight while the current one is
// reduced). Header fields are extracted from the loaded chunks with cross-lane shuffles and
// v_alignbyte_b32, so no load depends on packet contents. Two region sums (IP header, transport
// part) per packet; each region starts at an even packet offset, so the packet's address parity
// decides the rotation of both.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "netcsum_device.h"
#include "netcsum_kernels.h"

namespace netcsum {

namespace {

constexpr uint32_t F_IP_OK = 0x01u, F_L4_OK = 0x02u, F_L4_CHECKED = 0x04u, F_UDP_NO_CSUM = 0x08u,
                   F_MALFORMED = 0x10u, F_FRAGMENT = 0x20u, F_L4_MALFORMED = 0x40u, F_EXT_HDR = 0x80u;

template <int K>
struct PktStage {
    u32x4     v[K];
    uint32_t  lead;      // packet start offset inside its first 16-B chunk
    uint32_t  avail;     // bytes of the packet present in the buffer
    uintptr_t a;         // packet start address
};

// Pins a stage's loaded chunks behind everything issued before this point (an empty asm with a
// memory clobber that reads and writes them): the consume of the stage cannot be hoisted into the
// next stage's issue, so the wave issues all K loads of the next stage before it waits for this one
// (the Tx instantiation otherwise stalled on `s_waitcnt vmcnt(8)` between its issue loads).
template <int K>
__device__ __forceinline__ void pin_chunks(u32x4 (&v)[K]) {
#pragma unroll
    for (int k = 0; k < K; ++k) {
        asm volatile("" : "+v"(v[k]) : : "memory");
    }
}

// The packet's frame starts at the 16-B boundary below it; chunk c of the frame is
// [q0 + 16c, q0 + 16c + 16).
template <int G, int K, bool NT>
__device__ __forceinline__ void pkt_issue(PktStage<K>& st, uintptr_t a, uint32_t avail, int lane) {
    st.a = a;
    st.lead = (uint32_t)(a & 15u);
    st.avail = avail;
    const uintptr_t q0 = a - st.lead;
    const uint32_t nch = (avail + st.lead + 15u) >> 4;
    const uintptr_t z = zero_addr();
#pragma unroll
    for (int k = 0; k < K; ++k) {
        const uint32_t c = (uint32_t)(k * G + lane);
        gu32x4* src = reinterpret_cast<gu32x4*>((c < nch) ? (q0 + 16u * (uintptr_t)c) : z);
        st.v[k] = load16<NT>(src);
    }
}

__device__ __forceinline__ uint32_t pick4(u32x4 v, uint32_t comp) {
    uint32_t r = v.x;
    r = (comp == 1u) ? v.y : r;
    r = (comp == 2u) ? v.z : r;
    r = (comp == 3u) ? v.w : r;
    return r;
}

// Little-endian dword at packet offset i (lead + i + 7 < 16*G: the bytes sit in chunk slot 0 of
// the group's lanes). All lanes of the group get the same value.
__device__ __forceinline__ uint32_t pkt_dword(u32x4 v0, uint32_t lead, uint32_t i, int gbase) {
    const uint32_t r = lead + i;
    const uint32_t t = r >> 2;
    const uint32_t lo = (uint32_t)__shfl((int)pick4(v0, t & 3u), gbase + (int)(t >> 2), 64);
    const uint32_t hi = (uint32_t)__shfl((int)pick4(v0, (t + 1u) & 3u), gbase + (int)((t + 1u) >> 2), 64);
    const uint32_t b = r & 3u;
    return b ? __builtin_amdgcn_alignbyte(hi, lo, b) : lo;
}

__device__ __forceinline__ uint32_t be16_at(uint32_t dw, int byte) {   // bytes byte, byte+1 of dw, BE
    return (((dw >> (8 * byte)) & 0xFFu) << 8) | ((dw >> (8 * byte + 8)) & 0xFFu);
}

// What frame byte f adds to this lane's unfolded v_sad_u16 accumulator, read from the lane's OWN
// k = 0 chunk (0 unless the lane holds the byte; weight 2^(8(f&1)) in the absolute LE frame). Tx
// checksum fields count as zero: their bytes are subtracted where they were summed, with no
// cross-lane traffic (the transport field's offset depends on the IP header length, so a shuffle
// would add a dependent LDS round trip per packet).
__device__ __forceinline__ uint32_t own_byte(u32x4 v0, uint32_t f, int lane) {
    const uint32_t b = (pick4(v0, (f >> 2) & 3u) >> (8u * (f & 3u))) & 0xFFu;
    return ((uint32_t)lane == (f >> 4)) ? (b << (8u * (f & 1u))) : 0u;
}

struct PktInfo {
    uint32_t flags;
    uint32_t hlen;         // IPv4: IP header length. IPv6: bytes before the transport sum's start
                           // (8: the addresses open the sum; 40: ICMPv6 errors summed without pseudo)
    uint32_t l4_end;       // packet offset one past the transport part
    uint32_t l4_csum_off;  // packet offset of the transport checksum field (~0u: none)
    uint32_t ext_end;      // IPv6: packet offset of the transport header (40 + extension headers)
    uint32_t pseudo_le;    // little-endian word sum of the pseudo-header (0: none)
    uint32_t proto;
    bool     check_l4;
};

__device__ __forceinline__ uint32_t swap16(uint32_t x) { return ((x & 0xFFu) << 8) | ((x >> 8) & 0xFFu); }

// IPv6 (40-B fixed header, RFC 8200): no header checksum; the transport sums take the 40-B
// pseudo-header {src, dst, upper-layer length (32 bit), 0, next header} of net_ipv6.h:844-852.
// The addresses are packet bytes [8, 40), contiguous with the transport part, so the transport sum
// runs over [8, end) and only the length and next-header words are added in registers.
//   TCP (6)      DataVerify / DataCalc + pseudo                     net_tcp.c:7871-7879, 29839-29850
//   UDP (17)     as IPv4: 0 = no checksum (Rx), 0 -> 0xFFFF (Tx)    net_udp.c:1947-1957, 2909-2931
//   ICMPv6 (58)  Rx: types 1, 3, 4 (destination unreachable, time exceeded, parameter problem)
//                    HdrVerify over the message WITHOUT the pseudo-header  net_icmpv6.c:2910-2920
//                    types 128-131, 134-137 (echo, MLD, NDP) DataVerify + pseudo  net_icmpv6.c:2923-2942
//                    other types: rejected before any checksum (INVALID_TYPE)     net_icmpv6.c:2945-2948
//                Tx: every message through the pseudo-header (DataCalc + pseudo, net_icmpv6.c:1439;
//                    the error messages' ~HdrCalc(pseudo) field trick, net_icmpv6.c:949-965, gives
//                    the same value), no 0 -> 0xFFFF substitution
// Extension headers (net_ipv6.c:8290-8360, RxPktProcessExtHdr): Routing headers (43) the reference
// accepts (type <= 2 or Segments Left 0, net_ipv6.c:8735-8753) — length (HdrExtLen + 1) * 8,
// net_ipv6.c:8601 — are skipped, up to 4 of them, while the chain and the transport fields stay
// inside the bytes the group's first chunks hold (16 * G from the frame start); the transport part
// then starts after them and the pseudo-header length is the payload length minus their bytes
// (IP_DatagramLen = IP_TotLen - IPv6_ExtHdrLen, net_ipv6.c:5682). A Fragment header (44) means
// FRAGMENT: the transport checksum covers the reassembled datagram. Hop-by-Hop / Destination Options
// headers (whose options must be walked, net_ipv6.c:8604-8672), any other routing header, a chain
// past that window, and every other extension header (AH, ESP, Mobility, No Next Header,
// experimental values) get EXT_HDR here; the walk pass (netcsum_v6walk.hip) then judges each of
// those datagrams by the reference's rules; an extension header running past the payload is
// MALFORMED.
__device__ __forceinline__ bool ipv6_ext_hdr(uint32_t nh) {
    return nh == 0u || nh == 43u || nh == 44u || nh == 50u || nh == 51u || nh == 59u || nh == 60u ||
           nh == 135u || nh == 139u || nh == 140u || nh == 253u || nh == 254u;
}

template <int G, bool TX>
__device__ __forceinline__ PktInfo pkt_parse_v6(u32x4 v0, uint32_t lead, uint32_t avail, int gbase, uint32_t udp_mode,
                                                uint32_t d0, uint32_t d1) {   // packet dwords 0 and 1
    PktInfo p{};
    p.l4_csum_off = ~0u;
    const uint32_t plen = be16_at(d1, 0);
    const uint32_t tot = 40u + plen;
    p.proto = (d1 >> 16) & 0xFFu;
    p.ext_end = 40u;
    if (avail < 40u || ((d0 >> 4) & 0xFu) != 6u || tot > avail) {
        p.flags = F_MALFORMED;
        p.l4_end = 0u;
        p.hlen = 0u;
        return p;
    }
    p.l4_end = tot;
    p.hlen = 8u;
    // window: transport fields up to off + 24 and the dword reads below stay in the k = 0 chunks
    constexpr uint32_t kWin = 16u * (uint32_t)G;
    uint32_t off = 40u;
    // accepted Routing headers walked here; option headers and rejected-looking Routing headers go
    // to the walk pass (netcsum_v6walk.hip), which applies NetIPv6_RxOptHdr / RxRoutingHdr's rules
    for (int e = 0; e < 4 && p.proto == 43u; ++e) {
        if (lead + off + 8u > kWin) {
            p.flags |= F_EXT_HDR;
            return p;
        }
        const uint32_t d = pkt_dword(v0, lead, off, gbase);
        if (((d >> 16) & 0xFFu) > 2u && (d >> 24) != 0u) {
            p.flags |= F_EXT_HDR;
            return p;
        }
        off += (((d >> 8) & 0xFFu) + 1u) * 8u;
        p.proto = d & 0xFFu;
        if (off > tot) {
            p.flags = F_MALFORMED;
            p.l4_end = 0u;
            p.hlen = 0u;
            return p;
        }
    }
    if (p.proto == 44u) {
        p.flags |= F_FRAGMENT;
        return p;
    }
    if (ipv6_ext_hdr(p.proto) || (off != 40u && lead + off + 24u > kWin)) {
        p.flags |= F_EXT_HDR;
        return p;
    }
    p.ext_end = off;
    const uint32_t ulen = tot - off;                             // upper-layer packet length
    const uint32_t pseudo = (p.proto << 8) + swap16(ulen);       // length high half is 0 (< 2^16)
    switch (p.proto) {
    case 6u:
        if (ulen < 20u) {
            p.flags |= F_L4_MALFORMED;
            return p;
        }
        p.check_l4 = true;
        p.l4_csum_off = off + 16u;
        p.pseudo_le = pseudo;
        break;
    case 17u: {
        if (ulen < 8u) {
            p.flags |= F_L4_MALFORMED;
            return p;
        }
        const uint32_t du = pkt_dword(v0, lead, off + 4u, gbase);
        if (be16_at(du, 0) != ulen) {                            // net_udp.c:1903-1907
            p.flags |= F_L4_MALFORMED;
            return p;
        }
        p.l4_csum_off = off + 6u;
        if (!TX && (du >> 16) == 0u) {
            p.flags |= F_UDP_NO_CSUM | F_L4_OK;
            return p;
        }
        if (TX && !udp_tx_compute(udp_mode, du >> 16)) {
            p.flags |= F_UDP_NO_CSUM;
            return p;
        }
        p.check_l4 = true;
        p.pseudo_le = pseudo;
        break;
    }
    case 58u:
        if (ulen < 4u) {
            p.flags |= F_L4_MALFORMED;
            return p;
        }
        p.l4_csum_off = off + 2u;
        if constexpr (TX) {
            p.check_l4 = true;
            p.pseudo_le = pseudo;
        } else {
            const uint32_t type = pkt_dword(v0, lead, off, gbase) & 0xFFu;
            if (type == 1u || type == 3u || type == 4u) {
                p.check_l4 = true;
                p.hlen = off;                                    // message alone, no pseudo-header
            } else if ((type >= 128u && type <= 131u) || (type >= 134u && type <= 137u)) {
                p.check_l4 = true;
                p.pseudo_le = pseudo;
            }
        }
        break;
    default:
        break;
    }
    return p;
}

template <bool TX>
__device__ __forceinline__ PktInfo pkt_parse(u32x4 v0, uint32_t lead, uint32_t avail, int gbase, uint32_t udp_mode,
                                             uint32_t d0, uint32_t d1) {      // packet dwords 0 and 1
    PktInfo p{};
    p.l4_csum_off = ~0u;
    const uint32_t d2 = pkt_dword(v0, lead, 8u, gbase);
    const uint32_t d3 = pkt_dword(v0, lead, 12u, gbase);
    const uint32_t d4 = pkt_dword(v0, lead, 16u, gbase);
    const uint32_t ver = (d0 >> 4) & 0xFu;
    p.hlen = (d0 & 0xFu) * 4u;
    const uint32_t tot = be16_at(d0, 2);
    const uint32_t frag = be16_at(d1, 2) & 0x3FFFu;              // MF | fragment offset
    p.proto = (d2 >> 8) & 0xFFu;
    if (avail < 20u || ver != 4u || p.hlen < 20u || tot < p.hlen || tot > avail) {
        p.flags = F_MALFORMED;
        p.l4_end = 0u;
        p.hlen = 0u;
        return p;
    }
    p.l4_end = tot;
    if (frag != 0u) {
        p.flags |= F_FRAGMENT;
        return p;
    }
    const uint32_t l4len = tot - p.hlen;
    const uint32_t src_dst = __builtin_amdgcn_sad_u16(d3, 0u, __builtin_amdgcn_sad_u16(d4, 0u, 0u));
    switch (p.proto) {
    case 6u:                                                     // TCP: length = IP datagram length
        if (l4len < 20u) {
            p.flags |= F_L4_MALFORMED;
            return p;
        }
        p.check_l4 = true;
        p.l4_csum_off = p.hlen + 16u;
        p.pseudo_le = src_dst + (6u << 8) + (((l4len & 0xFFu) << 8) | (l4len >> 8));
        break;
    case 17u: {                                                  // UDP
        if (l4len < 8u) {
            p.flags |= F_L4_MALFORMED;
            return p;
        }
        const uint32_t du = pkt_dword(v0, lead, p.hlen + 4u, gbase);
        const uint32_t udp_len = be16_at(du, 0);
        if (udp_len != l4len) {                                  // net_udp.c:1903-1907 (also < 8)
            p.flags |= F_L4_MALFORMED;
            return p;
        }
        p.l4_csum_off = p.hlen + 6u;
        if (!TX && (du >> 16) == 0u) {                           // no checksum transmitted
            p.flags |= F_UDP_NO_CSUM | F_L4_OK;
            return p;
        }
        if (TX && !udp_tx_compute(udp_mode, du >> 16)) {
            p.flags |= F_UDP_NO_CSUM;                            // write 0 (NET_UDP_HDR_CHK_SUM_NONE)
            p.check_l4 = false;
            return p;
        }
        p.check_l4 = true;
        p.pseudo_le = src_dst + (17u << 8) + (((udp_len & 0xFFu) << 8) | (udp_len >> 8));
        break;
    }
    case 1u:                                                     // ICMPv4, no pseudo-header
    case 2u:                                                     // IGMP
        if (l4len < 4u) {
            p.flags |= F_L4_MALFORMED;
            return p;
        }
        p.check_l4 = true;
        p.l4_csum_off = p.hlen + 2u;
        break;
    default:
        break;
    }
    return p;
}

template <int G>
__device__ __forceinline__ void store_csum(uintptr_t a, uint32_t off, uint32_t host_val) {
    // global (not flat) stores: a flat store counts in lgkmcnt too and makes the waitcnt pass
    // drain vmcnt(0) in the next stage's issue. memcpy of the host-order value.
    __attribute__((address_space(1))) uint8_t* p = (__attribute__((address_space(1))) uint8_t*)(a + off);
    p[0] = (uint8_t)(host_val & 0xFFu);
    p[1] = (uint8_t)(host_val >> 8);
}

constexpr uint32_t kOOB = 0xFFFFFFFFu;     // buffer offset at/after every num_records: store dropped
constexpr int kRsrcWord3 = 0x00020000;     // gfx9-family raw buffer V# word 3

__device__ __forceinline__ __amdgpu_buffer_rsrc_t byte_rsrc(const void* base, uint32_t bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, (int)bytes, kRsrcWord3);
}

__device__ __forceinline__ void store_byte(__amdgpu_buffer_rsrc_t r, uint32_t v, uint32_t off) {
    __builtin_amdgcn_raw_buffer_store_b8((uint8_t)(v & 0xFFu), r, (int)off, 0, 0);
}

// A packet's stores, deferred: the kernel issues them right AFTER the next stage's loads, so no
// wait for a stage's loads can also wait for the previous packet's stores (the VMEM counter retires
// in issue order). Measured (profiles/r1tx11_tx_sweep.jsonl): no change for Tx — its extra time over
// Rx is the 2 M scattered header writes themselves (Tx with the stores compiled out: 0.250 ms).
struct PktStore {
    uintptr_t a;       // packet address
    uint32_t  vals;    // Tx: IP checksum | transport checksum << 16 (host order)
    uint32_t  meta;    // Tx: transport field offset, Rx: action | flags << 16 | store IP << 24 | store L4 << 25 |
                       // lane stores << 26
    uint32_t  idx;     // packet index (flags)
};

// BS (strided batches): every store is a raw buffer store executed by ALL lanes, the lanes that store
// nothing carrying an out-of-range offset, so every path issues the same VMEM stores and the
// compiler's vmcnt bookkeeping stays exact (stores under a lane-0 branch make it conservative).
template <int G, bool TX, bool BS>
__device__ __forceinline__ void pkt_store(const PktStore& ps, const PktBatchArgs& A) {
    const uint32_t f = (ps.meta >> 16) & 0xFFu;
    const bool me = (ps.meta >> 26) & 1u;
    if (me && (f & F_EXT_HDR) && A.defer_word != nullptr) {
        *A.defer_word = A.defer_tag;                             // the walk pass has work (benign race)
    }
    const bool si = TX && ((ps.meta >> 24) & 1u), sl = TX && ((ps.meta >> 25) & 1u);
    const uint32_t l4off = ps.meta & 0xFFFFu;
    if constexpr (BS) {
        // Packets of one stage lie within a few strides of the wave's lane-0 packet (the lowest
        // address of the stage; if lane 0 stores nothing, no lane does), so a V# based there
        // reaches them with 32-bit offsets.
        const uintptr_t wb = (((uintptr_t)__builtin_amdgcn_readfirstlane((uint32_t)(ps.a >> 32))) << 32) |
                             (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)ps.a);
        const uint32_t o = (uint32_t)(ps.a - wb);
        if constexpr (TX) {
            const __amdgpu_buffer_rsrc_t rp = byte_rsrc(reinterpret_cast<const void*>(wb), 0xFFFFFFFFu);
            store_byte(rp, ps.vals, si ? o + 10u : kOOB);        // memcpy of the host-order values
            store_byte(rp, ps.vals >> 8, si ? o + 11u : kOOB);
            store_byte(rp, ps.vals >> 16, sl ? o + l4off : kOOB);
            store_byte(rp, ps.vals >> 24, sl ? o + l4off + 1u : kOOB);
        }
        const __amdgpu_buffer_rsrc_t rf = byte_rsrc(A.flags_out, A.flags_out ? A.n : 0u);
        store_byte(rf, f, me ? ps.idx : kOOB);
        if constexpr (TX) {                                      // host-memory forms: what was written
            const uint64_t qb = A.fieldpos_out ? (uint64_t)A.n * 4u : 0u;
            const __amdgpu_buffer_rsrc_t rq = byte_rsrc(A.fieldpos_out, (uint32_t)(qb < 0xFFFFFFFFull ? qb : 0xFFFFFFFFull));
            __builtin_amdgcn_raw_buffer_store_b32((si ? kFieldIP : 0u) | (sl ? kFieldL4 | l4off : 0u), rq,
                                                  (int)(me ? ps.idx * 4u : kOOB), 0, 0);
        }
        if constexpr (!TX) {
            const __amdgpu_buffer_rsrc_t ra = byte_rsrc(A.action_out, A.action_out ? A.n : 0u);
            store_byte(ra, l4off, me ? ps.idx : kOOB);
        }
    } else {
        if (!me) {
            return;
        }
        if (si) {
            store_csum<G>(ps.a, 10u, ps.vals & 0xFFFFu);
        }
        if (sl) {
            store_csum<G>(ps.a, l4off, ps.vals >> 16);
        }
        if (A.flags_out) {
            A.flags_out[ps.idx] = (uint8_t)f;
        }
        if (!TX && A.action_out) {
            A.action_out[ps.idx] = (uint8_t)l4off;
        }
        if (TX && A.fieldpos_out) {
            A.fieldpos_out[ps.idx] = (si ? kFieldIP : 0u) | (sl ? kFieldL4 | l4off : 0u);
        }
    }
}

template <int G, int K, bool NT, bool TX, int VER>
__device__ __forceinline__ PktStore pkt_consume(const PktStage<K>& st, const PktBatchArgs& A, uint32_t idx, bool valid,
                                                int lane, int gbase) {
    // One sum over [lead, lead + end) (end = transport end, or the IP header end when the transport
    // part is not checked), plus the IP header alone from the k = 0 chunks (lead + hlen < 16*G).
    // Both are exact integer sums of the same frame half-words, so the transport part is their
    // difference — exact, hence still zero iff all its bytes are zero (the reference's all-zero ->
    // 0 / 0xFFFF distinction). TX checksum fields count as zero: their bytes are subtracted from
    // the owning lane's sums.
    //
    // The chunks are summed UNMASKED (chunks past `end` dropped by a select on their sum); the bytes
    // of the frame before the packet and those past `end` in the last chunk are subtracted once per
    // lane afterwards (low_bytes), instead of masking every chunk: the packet kernels are VALU-issue
    // bound (profiles/r1txp_pmc.json), and per-chunk edge masks executed on every k slot dominated.
    const uint32_t lead = st.lead;
    // VER 4 / 6: one IP version per batch; VER 0: per packet by the version nibble (a mixed NIC ring)
    // (the first two dwords, read once, outside the per-version branch)
    const uint32_t d0 = pkt_dword(st.v[0], lead, 0u, gbase);
    const uint32_t d1 = pkt_dword(st.v[0], lead, 4u, gbase);
    const bool is6 = (VER == 6) || (VER == 0 && ((d0 >> 4) & 0xFu) == 6u);
    PktInfo p = is6 ? pkt_parse_v6<G, TX>(st.v[0], lead, st.avail, gbase, A.udp_tx_csum, d0, d1)
                   : pkt_parse<TX>(st.v[0], lead, st.avail, gbase, A.udp_tx_csum, d0, d1);
    const uint32_t end = p.check_l4 ? p.l4_end : p.hlen;
    const uint32_t rend = lead + end;
    const uint32_t nch = (rend + 15u) >> 4;
    const uint32_t cl = nch - 1u;                                // chunk holding byte rend - 1 (~0u: none)
    uint32_t acc = 0u;
    u32x4 vl = u32x4{0u, 0u, 0u, 0u};                            // that chunk, on the lane holding it
#pragma unroll
    for (int k = 0; k < K; ++k) {
        // Every loaded register is consumed on every path (no branch: a load left unconsumed on some
        // path stays "pending" across the loop back-edge and the compiler drains vmcnt(0) there).
        const uint32_t c = (uint32_t)(k * G + lane);
        const u32x4 v = st.v[k];
        const uint32_t sv = sum4(v, 0u);
        acc += (c < nch) ? sv : 0u;
        vl.x = (c == cl) ? v.x : vl.x;
        vl.y = (c == cl) ? v.y : vl.y;
        vl.z = (c == cl) ? v.z : vl.z;
        vl.w = (c == cl) ? v.w : vl.w;
    }
    const int l16 = 16 * lane;
    const uint32_t pre = low_bytes(st.v[0], (int)lead - l16);   // frame bytes before the packet
    acc -= pre + (sum4(vl, 0u) - low_bytes(vl, (int)(rend - 16u * cl)));
    const uint32_t ip_raw = low_bytes(st.v[0], (int)(lead + p.hlen) - l16) - pre;
    if (nch > (uint32_t)(G * K)) {                               // packets longer than one pass
        const uintptr_t q0 = st.a - lead;
        for (uint32_t c0 = (uint32_t)(G * K); c0 < nch; c0 += (uint32_t)(G * K)) {
            u32x4 w[K];
#pragma unroll
            for (int k = 0; k < K; ++k) {
                const uint32_t c = c0 + (uint32_t)(k * G + lane);
                w[k] = load16<NT>(reinterpret_cast<gu32x4*>((c < nch) ? (q0 + 16u * (uintptr_t)c) : zero_addr()));
            }
#pragma unroll
            for (int k = 0; k < K; ++k) {
                const uint32_t c = c0 + (uint32_t)(k * G + lane);
                u32x4 v = w[k];                                  // zero chunk past the range
                if (c < nch) {
                    v = edge_mask_rel(v, c, lead, rend);
                }
                acc = sum4(v, acc);
            }
        }
    }
    uint32_t acc_ip = ip_raw, acc_l4 = acc - ip_raw;
    if (is6 && p.ext_end > 40u && p.hlen == 8u) {                 // addresses + transport, not the ext headers
        acc_l4 -= low_bytes(st.v[0], (int)(lead + p.ext_end) - l16) - low_bytes(st.v[0], (int)(lead + 40u) - l16);
    }
    if (TX) {
        if (!is6 && !(p.flags & F_MALFORMED)) {
            acc_ip -= own_byte(st.v[0], lead + 10u, lane) + own_byte(st.v[0], lead + 11u, lane);
        }
        if (p.check_l4) {
            const uint32_t f = lead + p.l4_csum_off;
            acc_l4 -= own_byte(st.v[0], f, lane) + own_byte(st.v[0], f + 1u, lane);
        }
    }
    uint32_t sip = fold16(acc_ip), sl4 = fold16(acc_l4);
    if (lead & 1u) {                                              // both regions start at even offsets
        sip = rot8(sip);
        sl4 = rot8(sl4);
    }
    sip = fold16(group_sum<G>(sip));
    sl4 = fold16(group_sum<G>(sl4) + p.pseudo_le);
    uint32_t f = p.flags;
    uint32_t cip = ~0u, cl4 = ~0u;                               // Tx values to store; ~0u = none
    if (!(f & F_MALFORMED)) {
        if constexpr (!TX) {
            f |= (is6 || sip == 0xFFFFu) ? F_IP_OK : 0u;          // IPv6: well-formed (no header checksum)
            if (p.check_l4) {
                f |= F_L4_CHECKED | ((sl4 == 0xFFFFu) ? F_L4_OK : 0u);
            }
        } else {
            if (!is6) {
                cip = (~sip) & 0xFFFFu;                          // net_ipv4.c:9578-9586
            }
            f |= F_IP_OK;
            if (p.check_l4) {
                cl4 = (~sl4) & 0xFFFFu;
                if (p.proto == 17u && cl4 == 0u) {
                    cl4 = 0xFFFFu;                               // RFC 768 (net_udp.c:2929-2931)
                }
                f |= F_L4_CHECKED | F_L4_OK;
            } else if ((f & F_UDP_NO_CSUM) && p.l4_csum_off != ~0u) {
                cl4 = 0u;                                        // no UDP checksum (net_udp.c:2935)
            }
        }
    }
    PktStore ps;
    ps.a = st.a;
    ps.vals = (cip & 0xFFFFu) | ((cl4 & 0xFFFFu) << 16);
    const uint32_t low = TX ? (p.l4_csum_off & 0xFFFFu) : rx_action(f, p.proto, is6, A.rx_cfg);
    ps.meta = low | ((f & 0xFFu) << 16) | (cip != ~0u ? 1u << 24 : 0u) |
              (cl4 != ~0u ? 1u << 25 : 0u) | ((valid && lane == 0) ? 1u << 26 : 0u);
    ps.idx = idx;
    return ps;
}

template <bool VARLEN>
__device__ __forceinline__ void pkt_desc(const PktBatchArgs& A, uint32_t i, uint64_t& off, uint32_t& avail) {
    if constexpr (VARLEN) {
        const uint32_t ic = (i < A.n) ? i : 0u;
        off = A.off[ic];
        avail = A.len[ic];
    } else {
        off = (uint64_t)i * A.stride;
        avail = A.len_u;
    }
}

// 4 waves per SIMD: the Tx instantiations otherwise take 131 VGPRs (3 waves), 25 % less memory
// parallelism than Rx (122 VGPRs); capped at 128 they do not spill (profiles/r1txp_pmc.json).
template <int G, int K, bool VARLEN, bool NT, bool TX, int VER>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(4))) pkt_batch_kernel(PktBatchArgs A) {
    static_assert(G >= 8, "header extraction needs the first 6 chunks in slot 0");
    const int lane = (int)(threadIdx.x & (G - 1));
    const int gbase = (int)(threadIdx.x & 63) & ~(G - 1);
    const uint32_t gpb = blockDim.x / G;
    const uint32_t grp = threadIdx.x / G;
    uint32_t first, step, end;
    if (A.tile) {
        const uint64_t t0 = (uint64_t)blockIdx.x * gpb * A.tile;
        first = (uint32_t)t0 + grp;
        step = gpb;
        end = (uint32_t)min<uint64_t>(t0 + (uint64_t)gpb * A.tile, A.n);
    } else {
        first = blockIdx.x * gpb + grp;
        step = gridDim.x * gpb;
        end = A.n;
    }
    const uint32_t cnt = group_iters(first, step, end);
    const uint32_t iters = __builtin_amdgcn_readfirstlane(cnt);   // wave-uniform trip count
    if (iters == 0u) {
        return;
    }
    const uintptr_t base = (uintptr_t)A.base;
    const uintptr_t z = zero_addr();
    PktStage<K> S0, S1;
    uint64_t off;
    uint32_t avail;
    uint32_t i = first;
    bool v0 = cnt != 0u, v1 = false;
    pkt_desc<VARLEN>(A, i, off, avail);
    pkt_issue<G, K, NT>(S0, v0 ? base + off : z, v0 ? avail : 0u, lane);
    PktStore pend{z, 0u, 0u, 0u};                                // nothing to store yet
    for (uint32_t j = 0u; j < iters; j += 2u) {                  // one scalar exit (see seg_pipe_kernel)
        uint32_t nx = i + step;
        v1 = j + 1u < cnt;
        pkt_desc<VARLEN>(A, nx, off, avail);
        pkt_issue<G, K, NT>(S1, v1 ? base + off : z, v1 ? avail : 0u, lane);
        pkt_store<G, TX, !VARLEN>(pend, A);                      // previous packet's stores, after the loads
        pin_chunks<K>(S0.v);
        pend = pkt_consume<G, K, NT, TX, VER>(S0, A, i, v0, lane, gbase);
        i = nx;
        nx = i + step;
        v0 = j + 2u < cnt;
        pkt_desc<VARLEN>(A, nx, off, avail);
        pkt_issue<G, K, NT>(S0, v0 ? base + off : z, v0 ? avail : 0u, lane);
        pkt_store<G, TX, !VARLEN>(pend, A);
        pin_chunks<K>(S1.v);
        pend = pkt_consume<G, K, NT, TX, VER>(S1, A, i, v1, lane, gbase);
        i = nx;
    }
    pkt_store<G, TX, !VARLEN>(pend, A);
}

template <int G, int K, bool VARLEN, bool TX, int VER>
hipError_t launch_pkt_gk(const PktBatchArgs& a, const LaunchCfg& c, hipStream_t s) {
    const uint32_t gpb = 256u / G;
    int grid;
    if (a.tile) {
        const uint64_t per = (uint64_t)gpb * a.tile;
        grid = (int)(((uint64_t)a.n + per - 1u) / per);
    } else {
        grid = c.grid > 0 ? c.grid : (int)(((uint64_t)a.n + gpb - 1u) / gpb);
    }
    if (c.nt) {
        hipLaunchKernelGGL((pkt_batch_kernel<G, K, VARLEN, true, TX, VER>), dim3(grid), dim3(256), 0, s, a);
    } else {
        hipLaunchKernelGGL((pkt_batch_kernel<G, K, VARLEN, false, TX, VER>), dim3(grid), dim3(256), 0, s, a);
    }
    return hipGetLastError();
}

template <bool VARLEN, bool TX, int VER>
hipError_t launch_pkt_v(const PktBatchArgs& a, const LaunchCfg& c, hipStream_t s) {
    switch (c.group_lanes) {
    case 8:  return c.chunks_per_pass <= 4 ? launch_pkt_gk<8, 4, VARLEN, TX, VER>(a, c, s)
                                           : launch_pkt_gk<8, 8, VARLEN, TX, VER>(a, c, s);
    case 16: return c.chunks_per_pass <= 3 ? launch_pkt_gk<16, 3, VARLEN, TX, VER>(a, c, s)
                                           : launch_pkt_gk<16, 6, VARLEN, TX, VER>(a, c, s);
    case 32: return c.chunks_per_pass <= 3 ? launch_pkt_gk<32, 3, VARLEN, TX, VER>(a, c, s)
                                           : launch_pkt_gk<32, 6, VARLEN, TX, VER>(a, c, s);
    default: return launch_pkt_gk<64, 4, VARLEN, TX, VER>(a, c, s);
    }
}

template <int VER>
hipError_t launch_pkt_ver(const PktBatchArgs& a, const LaunchCfg& c, bool tx, hipStream_t s) {
    if (a.off) {
        return tx ? launch_pkt_v<true, true, VER>(a, c, s) : launch_pkt_v<true, false, VER>(a, c, s);
    }
    return tx ? launch_pkt_v<false, true, VER>(a, c, s) : launch_pkt_v<false, false, VER>(a, c, s);
}

}  // namespace

hipError_t launch_pkt_batch(const PktBatchArgs& a, const LaunchCfg& c, bool tx, int ip_ver, hipStream_t s) {
    switch (ip_ver) {
    case 4:  return launch_pkt_ver<4>(a, c, tx, s);
    case 6:  return launch_pkt_ver<6>(a, c, tx, s);
    default: return launch_pkt_ver<0>(a, c, tx, s);
    }
}

}  // namespace netcsum
