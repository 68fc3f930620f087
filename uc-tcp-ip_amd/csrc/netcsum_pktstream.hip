// netcsum_pktstream.hip — gfx950 "run stream" kernel for strided IPv4 packet batches (SURVEY §8(f)
// rows 1 and 4): fused Rx validation and Tx finalize, the same per-packet semantics as
// pkt_batch_kernel (netcsum_packets.hip, whose header lists the reference call sites), in the form
// of seg_stream_kernel (netcsum_stream.hip): a WAVE owns a run of consecutive packets and reads
// their bytes exactly once as 1-KiB pieces (every wave-instruction 8 whole aligned lines).
//
// Per run:
//  1. prologue, lane k = packet k of the run: the 96 bytes from the 16-B boundary below the
//     packet (6 x 16-B loads; the IPv4 header with options <= 60 B plus the transport fields at
//     <= hlen + 17) are parsed IN THE LANE — version / IHL / total length / fragment / protocol,
//     UDP length, the pseudo-header {src, dst, 0, proto, len} (net_tcp.c:7851-7857,
//     net_udp.c:1918-1934) — and the IP header's exact half-word sum [0, hlen) is taken from the
//     same registers. This overlaps the run's first D pieces in flight.
//  2. stream: per packet ONE scalar event at its transport end (`end` = total length, or hlen
//     when no transport verdict): the exact sum of [start, end) over the wave (prefix masks + DPP
//     wave_total), parked in lane k of a VGPR. The transport sum is that total minus the IP header
//     sum — exact integers, so zero iff all its bytes are zero (the reference's 0 / 0xFFFF rule).
//  3. vector epilogue, lane k = packet k: Tx subtracts the checksum fields (treated as zero,
//     net_ipv4.c:9573), folds, rotates odd packets, adds the pseudo-header, and derives the same
//     verdict flags / checksum values as pkt_consume; results are stored once per run: Rx flags as
//     one coalesced byte store, Tx checksum fields in place (host-order value memcpy'd,
//     net_ipv4.c:9586, net_tcp.c:29862, net_udp.c:2937).
//
// IPv6 (VER 6) and mixed rings (VER 0, per datagram by the version nibble) take the same form with
// the parse of pkt_parse_v6 (netcsum_packets.hip, whose header cites net_ipv6.c / net_icmpv6.c):
// no header checksum; the transport sum is the stream total minus the window's sum of [0, 8) and of
// the extension headers [40, transport start) — the addresses [8, 40) stay in, the length and next
// header words of the 40-B pseudo-header are added in registers; ICMPv6 types 1/3/4 on Rx subtract
// all of [0, transport start) (no pseudo-header, net_icmpv6.c:2910-2920). Hop-by-Hop / Routing /
// Destination Options headers are walked inside the lane's window: the first 96 - lead bytes of the
// datagram (lead = its address mod 16); a chain beyond it gets EXT_HDR, as the lane-group kernel's
// beyond its 16 G - lead bytes, and the walk pass (netcsum_v6walk.hip) finishes it.
//
// Domain (pkt_stream_supported): strided batches (stride >= pkt_len >= 64; gaps <= 64 B for the
// whole-span bounds 0 and 3, any gap for the live-piece bounds 1 and 2) and offset/length batches
// (bounds 1 and 2).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>
#include <atomic>

#include "../../include/netcsum_mi355x.h"
#include "netcsum_device.h"
#include "netcsum_kernels.h"
#include "netcsum_stream.h"
#include "netcsum_v6walk.h"

namespace netcsum {

namespace {

using namespace sv;

constexpr uint32_t kMaxRunPkts = 64u;     // packets per wave run: lane k = packet k

__device__ __forceinline__ uint32_t be16(uint32_t dw, int byte) {   // bytes byte, byte+1 of dw, BE
    return (((dw >> (8 * byte)) & 0xFFu) << 8) | ((dw >> (8 * byte + 8)) & 0xFFu);
}

// A window element as an opaque register value. Every select below picks between such values:
// a select between two LOADS of one array is folded by the optimiser into a load with a computed
// index, which moves the whole window to scratch memory (112 B per lane, per packet run).
__device__ __forceinline__ uint32_t ov(uint32_t x) {
    asm volatile("" : "+v"(x));
    return x;
}

// Little-endian dword at packet offset x (lead + x + 3 < 96, lead + x >= 16 * C0): the 16-B chunk
// holding byte lead + x and the next chunk's first dword by one select chain over chunks [C0, 6), then
// a 4-way dword pick and one alignbyte (alignbyte by 0 is the low dword). About 40 VALU, against
// about 75 for two 24-way dword selects over the window.
template <int C0>
__device__ __forceinline__ uint32_t pkt_dword_at(const u32x4 (&h)[6], uint32_t lead, uint32_t x) {
    const uint32_t r = lead + x, c = r >> 4, q = (r >> 2) & 3u;
    uint32_t a0 = ov(h[C0].x), a1 = ov(h[C0].y), a2 = ov(h[C0].z), a3 = ov(h[C0].w);
    uint32_t a4 = C0 < 5 ? ov(h[C0 + 1].x) : 0u;
#pragma unroll
    for (int k = C0 + 1; k < 6; ++k) {
        const bool m = c == (uint32_t)k;
        a0 = m ? ov(h[k].x) : a0;
        a1 = m ? ov(h[k].y) : a1;
        a2 = m ? ov(h[k].z) : a2;
        a3 = m ? ov(h[k].w) : a3;
        a4 = m ? (k < 5 ? ov(h[k < 5 ? k + 1 : 5].x) : 0u) : a4;
    }
    const uint32_t lo = q == 0u ? a0 : q == 1u ? a1 : q == 2u ? a2 : a3;
    const uint32_t hi = q == 0u ? a1 : q == 1u ? a2 : q == 2u ? a3 : a4;
    return __builtin_amdgcn_alignbyte(hi, lo, r & 3u);
}

// The same for a fixed offset X (a multiple of 4): only lead >> 2 varies, a 4-way select.
template <int X>
__device__ __forceinline__ uint32_t pkt_dword_fixed(const uint32_t (&wd)[24], uint32_t lead) {
    constexpr int B = X / 4;
    const uint32_t j = lead >> 2;
    const uint32_t w0 = ov(wd[B]), w1 = ov(wd[B + 1]), w2 = ov(wd[B + 2]), w3 = ov(wd[B + 3]), w4 = ov(wd[B + 4]);
    const uint32_t lo = j == 0u ? w0 : j == 1u ? w1 : j == 2u ? w2 : w3;
    const uint32_t hi = j == 0u ? w1 : j == 1u ? w2 : j == 2u ? w3 : w4;
    return __builtin_amdgcn_alignbyte(hi, lo, lead & 3u);
}

// What the 2 bytes of a checksum field (even packet offset; b0 first) add to an exact sum in the
// absolute little-endian frame of a packet starting at an odd / even address.
__device__ __forceinline__ uint32_t field_le(uint32_t b0, uint32_t b1, bool odd) {
    return odd ? ((b0 << 8) + b1) : (b0 + (b1 << 8));
}

struct LanePkt {          // lane k's packet after the prologue
    uint32_t flags;
    uint32_t end;         // packet offset one past the bytes the stream sums (0: none)
    uint32_t ip_sum;      // IPv4: exact half-word sum of the IP header [0, hlen) (absolute LE frame);
                          // IPv6: the bytes of [0, end) outside the transport sum (see the header)
    uint32_t fields;      // Tx: exact contribution of the checksum fields to be zeroed (IP | L4 sum)
    uint32_t l4_field;    // Tx: contribution of the transport field alone
    uint32_t pseudo_le;
    uint32_t l4_csum_off; // ~0u: none
    uint32_t proto;
    bool     check_l4;
    bool     malformed;
    bool     v6;
};

// Exact half-word sum of packet bytes [0, x) from the lane's window (lead + x <= 96).
__device__ __forceinline__ uint32_t win_prefix(const u32x4 (&h)[6], uint32_t lead, uint32_t x) {
    uint32_t s = 0u - low_bytes(h[0], (int)lead);
#pragma unroll
    for (int c = 0; c < 6; ++c) {
        s += low_bytes(h[c], min(max((int)(lead + x) - 16 * c, 0), 16));
    }
    return s;
}

// Adds packet-frame dword d to an exact half-word sum in the absolute little-endian frame: for a
// packet at an odd address the absolute half-words pair each byte with its packet-frame neighbour
// the other way round, so sel (pkt_frame_sel) swaps the bytes of each half-word first.
__device__ __forceinline__ uint32_t frame_sum(uint32_t d, uint32_t sel, uint32_t acc) {
    return __builtin_amdgcn_sad_u16(__builtin_amdgcn_perm(d, d, sel), 0u, acc);
}

__device__ __forceinline__ uint32_t pkt_frame_sel(bool odd) { return odd ? 0x02030001u : 0x03020100u; }

// Exact half-word sum of the window's bytes [lead, lead + x) (absolute frame; lead < 16, lead + x <= 96):
// the dwords below the end's dword by one compare each, the end's partial dword by a chunk select,
// less the lead's bytes.
__device__ __forceinline__ uint32_t win_range_sum(const u32x4 (&h)[6], uint32_t lead, uint32_t x) {
    const uint32_t e = lead + x, je = e >> 2;
    uint32_t s = 0u;
#pragma unroll
    for (int c = 0; c < 6; ++c) {
        s = __builtin_amdgcn_sad_u16(4u * c + 0u < je ? h[c].x : 0u, 0u, s);
        s = __builtin_amdgcn_sad_u16(4u * c + 1u < je ? h[c].y : 0u, 0u, s);
        s = __builtin_amdgcn_sad_u16(4u * c + 2u < je ? h[c].z : 0u, 0u, s);
        s = __builtin_amdgcn_sad_u16(4u * c + 3u < je ? h[c].w : 0u, 0u, s);
    }
    // dword je's low e & 3 bytes (e = 96: none, and chunk 5 stands in for the absent chunk 6)
    const uint32_t c = je >> 2, q = je & 3u;
    uint32_t a0 = ov(h[0].x), a1 = ov(h[0].y), a2 = ov(h[0].z), a3 = ov(h[0].w);
#pragma unroll
    for (int k = 1; k < 6; ++k) {
        const bool m = c >= (uint32_t)k;
        a0 = m ? ov(h[k].x) : a0;
        a1 = m ? ov(h[k].y) : a1;
        a2 = m ? ov(h[k].z) : a2;
        a3 = m ? ov(h[k].w) : a3;
    }
    const uint32_t de = q == 0u ? a0 : q == 1u ? a1 : q == 2u ? a2 : a3;
    s = __builtin_amdgcn_sad_u16(de & ((1u << (8u * (e & 3u))) - 1u), 0u, s);
    return s - low_bytes(h[0], (int)lead);
}

__device__ __forceinline__ uint32_t swap16(uint32_t x) { return ((x & 0xFFu) << 8) | ((x >> 8) & 0xFFu); }

// Extension-header values of pkt_parse_v6 (netcsum_packets.hip).
__device__ __forceinline__ bool ipv6_ext(uint32_t nh) {
    return nh == 0u || nh == 43u || nh == 44u || nh == 50u || nh == 51u || nh == 59u || nh == 60u ||
           nh == 135u || nh == 139u || nh == 140u || nh == 253u || nh == 254u;
}

// IPv6 parse of pkt_parse_v6 from the lane's own window (RFC 8200; net_ipv6.c:8290-8360, 8601,
// 5682; net_tcp.c:7871-7879; net_udp.c:1947-1957; net_icmpv6.c:2910-2948).
template <bool TX>
__device__ __forceinline__ LanePkt lane_parse6(const uint32_t (&wd)[24], const u32x4 (&h)[6], uint32_t lead,
                                               uint32_t avail, bool odd, uint32_t udp_mode, uint32_t d0, uint32_t d1) {
    LanePkt p{};
    p.l4_csum_off = ~0u;
    p.v6 = true;
    const uint32_t tot = 40u + be16(d1, 0);
    uint32_t nh = (d1 >> 16) & 0xFFu;
    if (avail < 40u || ((d0 >> 4) & 0xFu) != 6u || tot > avail) {
        p.flags = NETCSUM_PKT_MALFORMED;
        p.malformed = true;
        return p;
    }
    const uint32_t window = 96u - lead;                          // bytes of the datagram in the window
    uint32_t off = 40u;
    // Routing headers the reference accepts (type <= 2 or Segments Left 0, net_ipv6.c:8735-8753) are
    // walked here; Hop-by-Hop / Destination Options headers (whose options NetIPv6_RxOptHdr walks,
    // net_ipv6.c:8604-8672) and any other routing header go to the walk pass (EXT_HDR), which judges them.
    for (int e = 0; e < 4 && nh == 43u; ++e) {
        if (off + 8u > window) {
            p.flags = NETCSUM_PKT_EXT_HDR;
            return p;
        }
        const uint32_t d = pkt_dword_at<2>(h, lead, off);
        if (((d >> 16) & 0xFFu) > 2u && (d >> 24) != 0u) {
            p.flags = NETCSUM_PKT_EXT_HDR;
            return p;
        }
        off += (((d >> 8) & 0xFFu) + 1u) * 8u;
        nh = d & 0xFFu;
        if (off > tot) {                                         // extension header past the payload
            p.flags = NETCSUM_PKT_MALFORMED;
            p.malformed = true;
            return p;
        }
    }
    if (nh == 44u) {
        p.flags = NETCSUM_PKT_FRAGMENT;
        return p;
    }
    if (ipv6_ext(nh) || (off != 40u && off + 24u > window)) {
        p.flags = NETCSUM_PKT_EXT_HDR;
        return p;
    }
    p.proto = nh;
    const uint32_t ulen = tot - off;                             // upper-layer length (< 2^16)
    const uint32_t pseudo = (nh << 8) + swap16(ulen);
    bool nopseudo = false;
    switch (nh) {
    case 6u:
        if (ulen < 20u) {
            p.flags = NETCSUM_PKT_L4_MALFORMED;
            return p;
        }
        p.check_l4 = true;
        p.l4_csum_off = off + 16u;
        break;
    case 17u: {
        if (ulen < 8u) {
            p.flags = NETCSUM_PKT_L4_MALFORMED;
            return p;
        }
        const uint32_t du = pkt_dword_at<2>(h, lead, off + 4u);
        if (be16(du, 0) != ulen) {
            p.flags = NETCSUM_PKT_L4_MALFORMED;
            return p;
        }
        p.l4_csum_off = off + 6u;
        if (!TX && (du >> 16) == 0u) {
            p.flags = NETCSUM_PKT_UDP_NO_CSUM | NETCSUM_PKT_L4_OK;
            return p;
        }
        if (TX && !udp_tx_compute(udp_mode, du >> 16)) {
            p.flags = NETCSUM_PKT_UDP_NO_CSUM;
            return p;
        }
        p.check_l4 = true;
        break;
    }
    case 58u:
        if (ulen < 4u) {
            p.flags = NETCSUM_PKT_L4_MALFORMED;
            return p;
        }
        p.l4_csum_off = off + 2u;
        if constexpr (TX) {
            p.check_l4 = true;
        } else {
            const uint32_t type = pkt_dword_at<2>(h, lead, off) & 0xFFu;
            if (type == 1u || type == 3u || type == 4u) {
                p.check_l4 = true;
                nopseudo = true;                                 // message alone (net_icmpv6.c:2910-2920)
            } else if ((type >= 128u && type <= 131u) || (type >= 134u && type <= 137u)) {
                p.check_l4 = true;
            }
        }
        break;
    default:
        break;
    }
    if (p.check_l4) {
        p.end = tot;
        if (off == 40u && !nopseudo) {
            // the bytes before the addresses: the fixed header's first 8 B, from d0 / d1
            const uint32_t sel = pkt_frame_sel(odd);
            p.ip_sum = frame_sum(d0, sel, frame_sum(d1, sel, 0u));
        } else {                                                 // walked routing headers / ICMPv6 errors
            const uint32_t s_off = win_prefix(h, lead, off);
            p.ip_sum = nopseudo ? s_off : s_off - (win_prefix(h, lead, 40u) - win_prefix(h, lead, 8u));
        }
        p.pseudo_le = nopseudo ? 0u : pseudo;
        if constexpr (TX) {
            const uint32_t fd = pkt_dword_at<2>(h, lead, p.l4_csum_off);
            p.l4_field = field_le(fd & 0xFFu, (fd >> 8) & 0xFFu, odd);
        }
    }
    return p;
}

// IPv4 parse of pkt_parse (netcsum_packets.hip) from the lane's own window; `avail` bytes present.
template <bool TX>
__device__ __forceinline__ LanePkt lane_parse(const uint32_t (&wd)[24], const u32x4 (&h)[6], uint32_t lead,
                                              uint32_t avail, bool odd, uint32_t udp_mode) {
    LanePkt p{};
    p.l4_csum_off = ~0u;
    const uint32_t d0 = pkt_dword_fixed<0>(wd, lead);
    const uint32_t d1 = pkt_dword_fixed<4>(wd, lead);
    const uint32_t d2 = pkt_dword_fixed<8>(wd, lead);
    const uint32_t d3 = pkt_dword_fixed<12>(wd, lead);
    const uint32_t d4 = pkt_dword_fixed<16>(wd, lead);
    const uint32_t ver = (d0 >> 4) & 0xFu;
    uint32_t hlen = (d0 & 0xFu) * 4u;
    const uint32_t tot = be16(d0, 2);
    const uint32_t frag = be16(d1, 2) & 0x3FFFu;                 // MF | fragment offset
    p.proto = (d2 >> 8) & 0xFFu;
    if (avail < 20u || ver != 4u || hlen < 20u || tot < hlen || tot > avail) {
        p.flags = NETCSUM_PKT_MALFORMED;
        p.malformed = true;
        return p;                                                // end 0: nothing summed
    }
    // exact sum of the IP header [0, hlen): the 20-B base header from d0..d4; with options, from the
    // window (lead + hlen <= 75 < 96)
    if (hlen == 20u) {
        const uint32_t sel = pkt_frame_sel(odd);
        p.ip_sum = frame_sum(d0, sel, frame_sum(d1, sel, frame_sum(d2, sel, frame_sum(d3, sel, frame_sum(d4, sel, 0u)))));
    } else {
        uint32_t s = 0u - low_bytes(h[0], (int)lead);
#pragma unroll
        for (int c = 0; c < 5; ++c) {
            s += low_bytes(h[c], min(max((int)(lead + hlen) - 16 * c, 0), 16));
        }
        p.ip_sum = s;
    }
    p.fields = TX ? field_le((d2 >> 16) & 0xFFu, d2 >> 24, odd) : 0u;   // IP checksum field, offset 10
    p.end = hlen;
    if (frag != 0u) {
        p.flags = NETCSUM_PKT_FRAGMENT;
        return p;
    }
    const uint32_t l4len = tot - hlen;
    const uint32_t src_dst = __builtin_amdgcn_sad_u16(d3, 0u, __builtin_amdgcn_sad_u16(d4, 0u, 0u));
    const uint32_t fo = p.proto == 17u ? hlen + 4u : (p.proto == 6u ? hlen + 16u : hlen + 2u);
    const uint32_t fd = pkt_dword_at<1>(h, lead, fo);              // UDP: len | csum; TCP / ICMP / IGMP: csum
    switch (p.proto) {
    case 6u:
        if (l4len < 20u) {
            p.flags = NETCSUM_PKT_L4_MALFORMED;
            return p;
        }
        p.check_l4 = true;
        p.l4_csum_off = hlen + 16u;
        p.pseudo_le = src_dst + (6u << 8) + (((l4len & 0xFFu) << 8) | (l4len >> 8));
        p.l4_field = TX ? field_le(fd & 0xFFu, (fd >> 8) & 0xFFu, odd) : 0u;
        break;
    case 17u: {
        if (l4len < 8u) {
            p.flags = NETCSUM_PKT_L4_MALFORMED;
            return p;
        }
        const uint32_t udp_len = be16(fd, 0);
        if (udp_len != l4len) {                                  // net_udp.c:1903-1907
            p.flags = NETCSUM_PKT_L4_MALFORMED;
            return p;
        }
        p.l4_csum_off = hlen + 6u;
        if (!TX && (fd >> 16) == 0u) {                           // no checksum transmitted
            p.flags = NETCSUM_PKT_UDP_NO_CSUM | NETCSUM_PKT_L4_OK;
            return p;
        }
        if (TX && !udp_tx_compute(udp_mode, fd >> 16)) {
            p.flags = NETCSUM_PKT_UDP_NO_CSUM;                   // write 0 (NET_UDP_HDR_CHK_SUM_NONE)
            return p;
        }
        p.check_l4 = true;
        p.pseudo_le = src_dst + (17u << 8) + (((udp_len & 0xFFu) << 8) | (udp_len >> 8));
        p.l4_field = TX ? field_le((fd >> 16) & 0xFFu, fd >> 24, odd) : 0u;
        break;
    }
    case 1u:                                                     // ICMPv4 / IGMP: no pseudo-header
    case 2u:
        if (l4len < 4u) {
            p.flags = NETCSUM_PKT_L4_MALFORMED;
            return p;
        }
        p.check_l4 = true;
        p.l4_csum_off = hlen + 2u;
        p.l4_field = TX ? field_le(fd & 0xFFu, (fd >> 8) & 0xFFu, odd) : 0u;
        break;
    default:
        break;
    }
    if (p.check_l4) {
        p.end = tot;
    }
    return p;
}

__device__ __forceinline__ void store_field(uint8_t* p, uint32_t v) {    // memcpy of a host-order u16
    __attribute__((address_space(1))) uint8_t* q = (__attribute__((address_space(1))) uint8_t*)p;
    q[0] = (uint8_t)(v & 0xFFu);
    q[1] = (uint8_t)(v >> 8);
}

// REC (Tx only): instead of writing the checksum fields, write one PktTxRecord per packet (dense,
// coalesced); pkt_scatter_kernel then writes the fields in a pass of its own.
template <int VER, bool TX>
__device__ __forceinline__ LanePkt lane_parse_ver(const uint32_t (&wd)[24], const u32x4 (&h)[6], uint32_t lead,
                                                  uint32_t avail, bool odd, uint32_t udp_mode) {
    if constexpr (VER == 4) {
        return lane_parse<TX>(wd, h, lead, avail, odd, udp_mode);
    } else {
        const uint32_t d0 = pkt_dword_fixed<0>(wd, lead);
        const uint32_t d1 = pkt_dword_fixed<4>(wd, lead);
        if (VER == 6 || ((d0 >> 4) & 0xFu) == 6u) {
            return lane_parse6<TX>(wd, h, lead, avail, odd, udp_mode, d0, d1);
        }
        return lane_parse<TX>(wd, h, lead, avail, odd, udp_mode);
    }
}

// VER 4 / 6: one IP version per batch; VER 0: per datagram by the version nibble (a mixed ring).
//
// Which bytes are read (BND, NETCSUM_TUNE_PKT_BOUND). A NIC ring's slots are larger than most of its
// frames: 1518 / 1520-B pool buffers holding 40-B ACKs (Cfg/Template/net_dev_cfg.c:146-149, one NET_BUF
// per frame, Source/net_buf.h:595-598, the frame length per frame from the driver, IF/net_if.c:6593),
// or 2-KiB buffers whose present bytes the caller passes as pkt_len.
//   0  the round-3 form: every 1-KiB piece of the run's span, the first D issued with the parse's
//      loads (dense strided layouts only: gaps <= 64 B);
//   1  live pieces, the parse first: only the pieces holding summed bytes are loaded, each masked to
//      its live 64-B sectors (below);
//   2  live pieces, with the run's piece 0 (which holds the first datagram's start) loaded whole
//      while the parse runs;
//   3  live pieces, with the run's first D pieces loaded whole while the parse runs (dense strided
//      layouts: at most D KiB per run read past the summed bytes; the rest as 1).
// Live pieces. After the parse each lane marks its datagram's summed bytes [a, a + end) as 64-B
// sectors (the HBM access unit) in a per-wave bitmap in LDS (1024 bits: a run spans <= 63 KiB), by
// ds_or of whole-dword ranges. Piece q's 16 sectors are halfword q; lane l holds halfword l, and a
// ballot of their non-zero values gives the run's live pieces as one uniform 64-bit mask (one
// SALU find-first-set and clear per piece: the kernels are scalar-issue bound on sparse layouts,
// profiles/r4h_instmix.txt). The stream then pops live pieces in address order, skipping dead
// ones entirely (no load, no consume), and lane l of piece q loads its 16 B only if sector l / 4 of
// the piece's mask (one readlane) is set. The stream's sums only take differences of prefixes inside
// [start, end) ranges, so zero-filled (unloaded) bytes outside them change nothing. The consume walk
// clamps offsets below the piece to 0: a datagram with nothing to sum (malformed: end 0) may start in
// a skipped piece, and its event then falls in a later one with an empty range.
// The pop: s_ff1 of the run's live-piece mask, which always holds bit 63 (piece 63 is never live:
// kLiveReach), so the empty mask needs no test: the sentinel piece 63 has no live sector (nothing
// loaded) and lies past every datagram end (its consume takes any pending events). Piece offsets x
// inside a consume take their two partial-lane byte masks from a table (one scalar load instead of
// ~12 SALU building them).
constexpr uint64_t kSentinel = 1ull << 63;
constexpr uint32_t kDone = ~0u;                         // end of "the next packet" once the run is done
struct PrefixMasks {
    uint64_t m0, m1;
};
constexpr uint64_t prefix_lo(uint32_t k) { return k >= 8u ? ~0ull : (1ull << (8u * k)) - 1ull; }
constexpr uint64_t prefix_hi(uint32_t k) { return k <= 8u ? 0ull : (1ull << (8u * (k - 8u))) - 1ull; }
__constant__ PrefixMasks kPrefixMask[16] = {
    {prefix_lo(0), prefix_hi(0)},   {prefix_lo(1), prefix_hi(1)},   {prefix_lo(2), prefix_hi(2)},
    {prefix_lo(3), prefix_hi(3)},   {prefix_lo(4), prefix_hi(4)},   {prefix_lo(5), prefix_hi(5)},
    {prefix_lo(6), prefix_hi(6)},   {prefix_lo(7), prefix_hi(7)},   {prefix_lo(8), prefix_hi(8)},
    {prefix_lo(9), prefix_hi(9)},   {prefix_lo(10), prefix_hi(10)}, {prefix_lo(11), prefix_hi(11)},
    {prefix_lo(12), prefix_hi(12)}, {prefix_lo(13), prefix_hi(13)}, {prefix_lo(14), prefix_hi(14)},
    {prefix_lo(15), prefix_hi(15)}};

// piece_prefix (netcsum_stream.h) with the table's masks.
__device__ __forceinline__ uint32_t piece_prefix_t(u32x4 v, uint32_t s4, uint32_t lane16, uint32_t x) {
    const PrefixMasks m = kPrefixMask[x & 15u];
    uint32_t pv = __builtin_amdgcn_sad_u16(v.x & (uint32_t)m.m0, 0u, 0u);
    pv = __builtin_amdgcn_sad_u16(v.y & (uint32_t)(m.m0 >> 32), 0u, pv);
    pv = __builtin_amdgcn_sad_u16(v.z & (uint32_t)m.m1, 0u, pv);
    pv = __builtin_amdgcn_sad_u16(v.w & (uint32_t)(m.m1 >> 32), 0u, pv);
    return (lane16 + 16u <= x) ? s4 : ((lane16 < x) ? pv : 0u);
}
// One wave run: packets s_begin .. s_begin + nres - 1, lane k's packet at run-relative offset prel
// (from O, 128-B aligned) with `avail` bytes present; the run's bytes [O, O + span). VL: per-packet
// starts (offset/length descriptors) instead of a stride.
template <int D, bool NT, bool TX, bool REC, int VER, int BND, bool VL>
__device__ __forceinline__ void pkt_run(const PktBatchArgs& A, PktTxRecord* rec, uint32_t w, uint32_t lane,
                                        uint32_t s_begin, uint32_t nres, uintptr_t O, uint32_t prel, uint32_t avail,
                                        uint32_t span) {
    const uint32_t st = (uint32_t)A.stride;
    const uint32_t lead0 = (uint32_t)__builtin_amdgcn_readfirstlane((int)prel);
    const uint32_t npieces = (span + 1023u) >> 10;
    const __amdgpu_buffer_rsrc_t rd = run_rsrc(O, (span + 15u) & ~15u);
    const uint32_t lane16 = 16u * lane;

    u32x4 dv[D];
    constexpr int kSpec = BND == 0 || BND == 3 ? D : BND == 2 ? 1 : 0;   // pieces loaded before the parse
#pragma unroll
    for (int j = 0; j < kSpec; ++j) {                          // the first pieces in flight ...
        dv[j] = buf_load16<NT>(rd, ((uint32_t)j << 10) + lane16);
    }

    // ... while lane k parses packet k from its own 96-B window.
    const bool mine = lane < nres;
    const uint32_t plead = prel & 15u;
    const uint32_t pq = prel - plead;
    u32x4 h[6];
#pragma unroll
    for (int c = 0; c < 6; ++c) {
        h[c] = buf_load16<false>(rd, mine ? pq + 16u * (uint32_t)c : kOOB);
    }
    uint32_t wd[24];
#pragma unroll
    for (int c = 0; c < 6; ++c) {
        wd[4 * c] = h[c].x;
        wd[4 * c + 1] = h[c].y;
        wd[4 * c + 2] = h[c].z;
        wd[4 * c + 3] = h[c].w;
    }
    const bool odd = (prel & 1u) != 0u;                        // O is 128-B aligned
    const LanePkt pk = lane_parse_ver<VER, TX>(wd, h, plead, avail, odd, A.udp_tx_csum);
    const uint32_t end_v = mine ? pk.end : 0u;
    // Live forms: datagrams whose summed bytes lie inside the lane's window (40-B ACKs; nothing to
    // sum) are summed here from the window: the stream neither marks their sectors nor walks their
    // events. (Form 0, the packed layouts, keeps every datagram in the stream: enabled there, the
    // window sum raised the VGPR count of the IPv6 offset/length kernels, which inline form 0.)
    const bool inwin = BND >= 1 ? plead + end_v <= 96u : end_v == 0u;
    uint32_t tot_v = 0u;                                       // packet k's [start, end) sum: lane k
    if (BND >= 1 && mine && inwin && end_v != 0u) {
        tot_v = win_range_sum(h, plead, end_v);
    }
    uint64_t srest = __builtin_amdgcn_ballot_w64(mine && !inwin);   // the stream's packets (lanes)
    // Row touch (off by default here: the header loads above already touch every datagram) issued
    // after the parse, when the window's registers are free (issued before it, its two VGPRs raised
    // the prologue's peak to 73 = 6 waves/SIMD).
    const RunTouch touch = touch_run(rd, npieces, lane, A.touch != 0u);
    uint64_t lm0 = 0u;                                         // live pieces of the run (<= 64)
    uint32_t pm0 = 0u;                                         // sector mask of piece `lane`
    uint32_t nlive = npieces;
    // Offset/length: a datagram past the bitmap's reach (a run of one, > 63 KiB from its 128-B line)
    // streams its whole span in order through the same piece ring (wide_stream below) — in this
    // instantiation, so the offset/length kernels carry no form-0 copy of the run (VERDICT r4 weak 4:
    // that copy and its 4 pieces loaded before the parse set their VGPR count).
    const bool wide = VL && BND >= 1 && span > kLiveReach;
    if (BND >= 1 && !wide) {
        __shared__ uint32_t sect_all[16][32];                   // (blocks of up to 16 waves)
        uint32_t* sect = sect_all[w];
        if (lane < 32u) {
            sect[lane] = 0u;
        }
        __builtin_amdgcn_wave_barrier();
        if (!inwin) {
            const uint32_t s0 = prel >> 6, s1 = (prel + end_v - 1u) >> 6;
            for (uint32_t d = s0 >> 5; d <= (s1 >> 5); ++d) {
                const uint32_t lo = max(s0, d << 5) - (d << 5), hi = min(s1, (d << 5) + 31u) - (d << 5);
                atomicOr(&sect[d], (2u << hi) - (1u << lo));   // bits lo..hi (hi = 31: 2 << 31 wraps to 0)
            }
        }
        __builtin_amdgcn_wave_barrier();
        pm0 = reinterpret_cast<const uint16_t*>(sect)[lane];
        lm0 = __builtin_amdgcn_ballot_w64(pm0 != 0u);
        nlive = (uint32_t)__builtin_popcountll(lm0);
    }
    const uint32_t lbit = 1u << (lane >> 2);                   // the lane's 64-B sector in a piece
    auto pop = [&]() -> uint32_t {                             // next live piece (uniform; none: 63)
        const uint32_t q = (uint32_t)__builtin_ctzll(lm0);     // (lm0 holds the sentinel)
        lm0 = (lm0 & (lm0 - 1u)) | kSentinel;
        return q;
    };
    auto live_voff = [&](uint32_t q) -> uint32_t {             // lane's offset in piece q, or OOB
        const uint32_t sm = (uint32_t)__builtin_amdgcn_readlane((int)pm0, (int)q);
        return (sm & lbit) ? (q << 10) + lane16 : kOOB;
    };
    uint32_t qd[D];                                            // the piece in flight in slot j
    if constexpr (BND >= 1) {
        // pieces 0 .. kSpec - 1 are in flight already: consumed first, whether live or not
        constexpr uint64_t spec = kSpec ? (1ull << kSpec) - 1u : 0u;
#pragma unroll
        for (int j = 0; j < kSpec; ++j) {
            qd[j] = (uint32_t)j;
        }
        if (!wide) {
            nlive = (uint32_t)__builtin_popcountll(lm0 | spec);
            lm0 = (lm0 & ~spec) | kSentinel;
#pragma unroll
            for (int j = kSpec; j < D; ++j) {
                qd[j] = pop();
                dv[j] = buf_load16<NT>(rd, live_voff(qd[j]));
            }
        } else {
#pragma unroll
            for (int j = kSpec; j < D; ++j) {
                qd[j] = (uint32_t)j;
                dv[j] = buf_load16<NT>(rd, ((uint32_t)j << 10) + lane16);
            }
        }
    }

    // The stream's next packet to finish (its lane; srest: the later ones) and its start / end,
    // run-relative; none: kDone.
    auto start_of = [&](uint32_t k) -> uint32_t {
        if constexpr (VL) {
            return (uint32_t)__builtin_amdgcn_readlane((int)prel, (int)k);
        } else {
            return lead0 + k * st;
        }
    };
    const bool any = srest != 0u;
    uint32_t cur = any ? (uint32_t)__builtin_ctzll(srest) : 63u;
    srest &= srest - 1u;
    uint32_t cs = start_of(cur);
    uint32_t ce = any ? cs + (uint32_t)__builtin_amdgcn_readlane((int)end_v, (int)cur) : kDone;
    uint32_t acc = 0u;

    // General walk of seg_stream_kernel with per-packet ends (state written back unconditionally).
    // Once the run's last packet has ended, e = kDone: no later piece has an event, and what the
    // walk accumulates is never used.
    auto consume = [&](uint32_t q, u32x4 v) {
        const uint32_t qb = q << 10;
        const uint32_t pend = qb + 1024u;
        const uint32_t full = sum4(v, 0u);
        uint32_t u = cur, c = cs, e = ce, a = acc, t = tot_v;
        uint64_t rs = srest;
        if (e > pend) {                                        // no packet ends in this piece
            a += (c <= qb) ? full : full - piece_prefix_t(v, full, lane16, min(c - qb, 1024u));
        } else {
            uint32_t Ps = (c <= qb) ? 0u : piece_prefix_t(v, full, lane16, c - qb);
#pragma clang loop vectorize(disable) unroll(disable)
            do {
                const uint32_t Pe = piece_prefix_t(v, full, lane16, e <= qb ? 0u : e - qb);
                const uint32_t T = wave_total(a + (Pe - Ps));
                t = (lane == u) ? T : t;
                a = 0u;
                const bool more = rs != 0u;
                u = more ? (uint32_t)__builtin_ctzll(rs) : 63u;
                rs &= rs - 1u;
                c = start_of(u);
                const bool adj = c == e;                       // dense: the next packet starts at this end
                e = more ? c + (uint32_t)__builtin_amdgcn_readlane((int)end_v, (int)u) : kDone;
                Ps = adj ? Pe : piece_prefix_t(v, full, lane16, c <= qb ? 0u : min(c - qb, 1024u));
            } while (e <= pend);
            a = full - Ps;
        }
        cur = u;
        srest = rs;
        cs = c;
        ce = e;
        acc = a;
        tot_v = t;
    };

    const uint32_t rounds = (nlive + (uint32_t)D - 1u) / (uint32_t)D;
    if (wide) {                                                // (VL only: every piece, in order)
        for (uint32_t r = 0; r < rounds; ++r) {
#pragma unroll
            for (int j = 0; j < D; ++j) {
                consume(qd[j], opaque_tuple(dv[j]));
                qd[j] += (uint32_t)D;
                dv[j] = buf_load16<NT>(rd, (qd[j] << 10) + lane16);             // past the run: zeros
                asm volatile("" ::: "memory");
            }
        }
    }
    for (uint32_t r = 0; r < (wide ? 0u : rounds); ++r) {
#pragma unroll
        for (int j = 0; j < D; ++j) {
            if constexpr (BND >= 1) {
                consume(qd[j], opaque_tuple(dv[j]));
                qd[j] = pop();                                                // none left: OOB, zeros
                dv[j] = buf_load16<NT>(rd, live_voff(qd[j]));
            } else {
                const uint32_t q = r * (uint32_t)D + (uint32_t)j;
                consume(q, opaque_tuple(dv[j]));
                dv[j] = buf_load16<NT>(rd, ((q + (uint32_t)D) << 10) + lane16);   // past the run: zeros
            }
            asm volatile("" ::: "memory");
        }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    touch_retire(touch);

    // IPv6 / mixed rings without a deferral word (Rx, and one-pass Tx): the wave finishes its own
    // deferred datagrams (EXT_HDR: chains past the window) after the epilogue, all 64 lanes together
    // (walk_wave). Two-pass Tx: the scatter pass walks them (pkt_scatter_kernel<WALK>).
    constexpr bool kWalkHere = !REC && VER != 4;
    const bool walk_here = kWalkHere && A.defer_word == nullptr;           // wave-uniform
    bool need = false;
    if (mine) {
    // vector epilogue: lane k = packet s_begin + k (pkt_consume's verdicts / values)
    uint32_t acc_ip = pk.ip_sum, acc_l4 = tot_v - pk.ip_sum;
    if (TX && !pk.malformed) {
        acc_ip -= pk.fields;
        if (pk.check_l4) {
            acc_l4 -= pk.l4_field;
        }
    }
    uint32_t sip = fold16(acc_ip), sl4 = fold16(acc_l4);
    if (odd) {
        sip = rot8(sip);
        sl4 = rot8(sl4);
    }
    sl4 = fold16(sl4 + pk.pseudo_le);
    uint32_t f = pk.flags;
    uint32_t cip = ~0u, cl4 = ~0u;
    if (!pk.malformed) {
        if constexpr (!TX) {
            f |= (pk.v6 || sip == 0xFFFFu) ? NETCSUM_PKT_IP_OK : 0u;   // IPv6: well-formed (no header checksum)
            if (pk.check_l4) {
                f |= NETCSUM_PKT_L4_CHECKED | ((sl4 == 0xFFFFu) ? NETCSUM_PKT_L4_OK : 0u);
            }
        } else {
            cip = pk.v6 ? ~0u : ((~sip) & 0xFFFFu);             // net_ipv4.c:9578-9586; IPv6: none
            f |= NETCSUM_PKT_IP_OK;
            if (pk.check_l4) {
                cl4 = (~sl4) & 0xFFFFu;
                if (pk.proto == 17u && cl4 == 0u) {
                    cl4 = 0xFFFFu;                               // RFC 768 (net_udp.c:2929-2931)
                }
                f |= NETCSUM_PKT_L4_CHECKED | NETCSUM_PKT_L4_OK;
            } else if ((f & NETCSUM_PKT_UDP_NO_CSUM) && pk.l4_csum_off != ~0u) {
                cl4 = 0u;                                        // no UDP checksum (net_udp.c:2935)
            }
        }
    }
    const uint32_t idx = s_begin + lane;
    need = walk_here && (f & NETCSUM_PKT_EXT_HDR) != 0u;               // walk_one writes its verdict
    if (A.defer_word != nullptr && (f & NETCSUM_PKT_EXT_HDR)) {
        *A.defer_word = A.defer_tag;                             // the walk pass has work (benign race)
    }
    if constexpr (REC) {
        // one 8-B store per packet (a struct assignment compiles to four partial stores, which
        // made this pass ~70 us slower on 1 M packets)
        const uint64_t r = (uint64_t)((cip & 0xFFFFu) | ((cl4 & 0xFFFFu) << 16)) |
                           ((uint64_t)(pk.l4_csum_off & 0xFFFFu) << 32) | ((uint64_t)(f & 0xFFu) << 48) |
                           ((uint64_t)((cip != ~0u ? 1u : 0u) | (cl4 != ~0u ? 2u : 0u)) << 56);
        reinterpret_cast<uint64_t*>(rec)[idx] = r;
    } else {
    if (A.flags_out && !need) {
        A.flags_out[idx] = (uint8_t)f;
    }
    if (!TX && A.action_out && !need) {
        A.action_out[idx] = (uint8_t)rx_action(f, pk.proto, pk.v6, A.rx_cfg);
    }
    if constexpr (TX) {
        uint8_t* p = reinterpret_cast<uint8_t*>(O + prel);
        if (cip != ~0u) {
            store_field(p + 10, cip);
        }
        if (cl4 != ~0u) {
            store_field(p + pk.l4_csum_off, cl4);
        }
        if (A.fieldpos_out && !need) {
            A.fieldpos_out[idx] = (cip != ~0u ? kFieldIP : 0u) | (cl4 != ~0u ? kFieldL4 | (pk.l4_csum_off & 0xFFFFu) : 0u);
        }
    }
    }
    }
    if constexpr (kWalkHere) {
        if (walk_here) {
            v6walk::walk_wave<TX>(A, s_begin, need, lane);
        }
    }
}

// Offset/length runs (VL) are streamed when their datagrams lie in increasing address order, each
// slot's present bytes ending before the next one starts, within 64 KiB from the run's first
// 128-B line (the live-piece bitmap's reach); any other run is done one datagram at a time, each as
// a run of its own (correct for any order or overlap, at one prologue per datagram).
// Run `run` (packets run * spw ...) by wave w of its block.
template <int D, bool NT, bool TX, bool REC, int VER, int BND, bool VL, bool DEFER = false>
__device__ __forceinline__ void pkt_stream_run(const PktBatchArgs& A, uint32_t spw, PktTxRecord* rec, uint64_t run,
                                               uint32_t w, uint32_t lane) {
    // (offset/length runs: the live-piece forms 1 / 2; a datagram past the bitmap's reach streams its
    // whole span inside them, pkt_run `wide`)
    static_assert(!VL || BND == 1 || BND == 2, "offset/length runs take the live-piece forms");
    const uint64_t sb64 = run * spw;
    if (sb64 >= A.n) {
        return;
    }
    const uint32_t s_begin = (uint32_t)sb64;
    const uint32_t nres = min(A.n - s_begin, spw);
    if constexpr (!VL) {
        const uintptr_t a_first = (uintptr_t)A.base + (uint64_t)s_begin * A.stride;
        const uintptr_t O = a_first & ~(uintptr_t)127;
        const uint32_t lead0 = (uint32_t)(a_first - O);
        const uint32_t st = (uint32_t)A.stride;
        pkt_run<D, NT, TX, REC, VER, BND, VL>(A, rec, w, lane, s_begin, nres, O, lead0 + lane * st, A.len_u,
                                             lead0 + (nres - 1u) * st + A.len_u);
    } else {
        const bool mine = lane < nres;
        const uint64_t off = A.off[mine ? s_begin + lane : s_begin];
        const uint32_t len = mine ? (uint32_t)A.len[s_begin + lane] : 0u;
        const uint64_t off0 = ((uint64_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(off >> 32)) << 32) |
                              (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)off);
        const uintptr_t O = ((uintptr_t)A.base + off0) & ~(uintptr_t)127;
        const uint64_t rel = (uintptr_t)A.base + off - O;                 // >= 0 when ordered
        const uint64_t end = rel + len;
        // ordered: lane k starts at or after lane k - 1's present bytes end (DPP shift by one lane)
        const uint32_t prev_end_lo = (uint32_t)__shfl_up((int)(uint32_t)end, 1, 64);
        const bool ok = !mine || (rel < kLiveReach && end <= kLiveReach - 128u &&
                                  (lane == 0u || (uint64_t)prev_end_lo <= rel));
        if (__builtin_amdgcn_ballot_w64(!ok) == 0u) {
            const uint32_t span = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)end, (int)(nres - 1u));
            pkt_run<D, NT, TX, REC, VER, BND, VL>(A, rec, w, lane, s_begin, nres, O, mine ? (uint32_t)rel : 0u,
                                                 len, span);
        } else if (DEFER) {
            // any other run (unordered, overlapping, far apart, or a datagram past the bitmap's reach)
            // is flagged for the deferred pass (pkt_vl_deferred_kernel): done here, one datagram at a
            // time, its loop held the offset/length kernels at 91-93 VGPRs (4-5 waves per SIMD;
            // VERDICT r4 weak 4), for the sake of layouts a NIC ring does not have. (One atomic add per
            // deferred run: appends by compare-and-swap on a tagged word took a batch of 32 768 deferred
            // runs 289 ms.)
            if (lane == 0u) {
                const uint32_t k = __hip_atomic_fetch_add(A.vl_ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                // the list holds one entry per run of this batch; a count left over by a failed call
                // is zeroed by the host before the next one (ScratchLease), so k stays below it —
                // checked anyway, since an entry past it would land outside the lease
                if ((uint64_t)k < ((uint64_t)A.n + spw - 1u) / spw) A.vl_list[k] = (uint32_t)run;
            }
        } else {
            // (the burst server, which has no deferred pass) one datagram per run (any order, overlap
            // or distance; a datagram past the bitmap's reach streams its whole span, pkt_run `wide`)
            for (uint32_t k = 0; k < nres; ++k) {
                const uint64_t ok_ = ((uint64_t)__builtin_amdgcn_readlane((int)(uint32_t)(off >> 32), (int)k) << 32) |
                                     (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)off, (int)k);
                const uint32_t lk = (uint32_t)__builtin_amdgcn_readlane((int)len, (int)k);
                const uintptr_t Ok = ((uintptr_t)A.base + ok_) & ~(uintptr_t)127;
                const uint32_t pk = (uint32_t)((uintptr_t)A.base + ok_ - Ok);
                pkt_run<D, NT, TX, REC, VER, BND, VL>(A, rec, w, lane, s_begin + k, 1u, Ok, pk, lk, pk + lk);
            }
        }
    }
}

// The deferred pass of an offset/length batch: the runs its stream kernel listed (A.vl_list, count in
// A.vl_ctr[0]), each in ordered sub-runs inside the reach, waves taking list entries round-robin; the
// last block to finish leaves the count and its own counter zero for the next batch on the stream.
// Launched after the stream kernel in stream order (and before two-pass Tx's scatter): 8 blocks when
// the ring's plan found its descriptors in order (a run listed anyway, e.g. where the ring wraps, is
// still done), one per 4 runs up to 2048 otherwise (the ring's first batch, reordered rings, runs
// asked for that outgrow the reach).
template <int D, bool NT, bool TX, bool REC, int VER, int BND>
__global__ void __launch_bounds__(256) pkt_vl_deferred_kernel(PktBatchArgs A, uint32_t spw, PktTxRecord* rec) {
    __shared__ uint32_t s_last;
    const uint32_t w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t runs = (uint32_t)(((uint64_t)A.n + spw - 1u) / spw);
    const uint32_t count = min(*A.vl_ctr, runs);
    // the blocks the list needs (4 entries each at first); the rest leave at once, touching nothing,
    // so the grid can be sized for a whole batch deferred at the cost of one load per idle block (a
    // block that reads the count after the reset below reads 0 and leaves too)
    const uint32_t active = min(gridDim.x, (count + 3u) / 4u);
    if (blockIdx.x >= active) {
        return;
    }
    for (uint32_t i = blockIdx.x * 4u + w; i < count; i += active * 4u) {
        const uint32_t r = A.vl_list[i];
        const uint32_t s_begin = r * spw;
        const uint32_t nres = r < runs ? min(A.n - s_begin, spw) : 0u;
        // the run in sub-runs: from datagram k0, the longest prefix in order and inside the reach of
        // k0's 128-B line streams as one wave run (a run that only outgrew the reach — runs of 32 in
        // 2-KiB slots — costs two streamed sub-runs, not 32 prologues); a datagram out of order, or
        // past the reach on its own, is a sub-run of one (`wide` in pkt_run)
        for (uint32_t k0 = 0; k0 < nres;) {
            const uint32_t idx = k0 + lane;
            const bool mine = idx < nres;
            const uint64_t off = A.off[s_begin + (mine ? idx : k0)];
            const uint32_t len = mine ? (uint32_t)A.len[s_begin + idx] : 0u;
            const uint64_t off0 = ((uint64_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(off >> 32)) << 32) |
                                  (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)off);
            const uintptr_t O = ((uintptr_t)A.base + off0) & ~(uintptr_t)127;
            const uint64_t rel = (uintptr_t)A.base + off - O;
            const uint64_t end = rel + len;
            const uint32_t prev_end_lo = (uint32_t)__shfl_up((int)(uint32_t)end, 1, 64);
            const bool ok = mine && rel < kLiveReach && end <= kLiveReach - 128u &&
                            (lane == 0u || (uint64_t)prev_end_lo <= rel);
            const uint64_t cut = ~__builtin_amdgcn_ballot_w64(ok);
            const uint32_t m = max(cut ? (uint32_t)__builtin_ctzll(cut) : 64u, 1u);
            const uint32_t span = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)end, (int)(m - 1u));
            const bool in = lane < m;
            pkt_run<D, NT, TX, REC, VER, BND, true>(A, rec, w, lane, s_begin + k0, m, O, in ? (uint32_t)rel : 0u,
                                                    in ? len : 0u, span);
            k0 += m;
        }
    }
    __syncthreads();
    if (threadIdx.x == 0u) {
        s_last = __hip_atomic_fetch_add(A.vl_ctr + 1, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT) == active - 1u;
        if (s_last) {                                           // every active block has read the count
            __hip_atomic_store(A.vl_ctr, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(A.vl_ctr + 1, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
}

// ---- the plan for the next batch on this ring (strided batches that are not packed)
// Which form reads a ring fastest depends on its frames' lengths, which the host cannot see in a
// device-resident batch (tools/ring_probe.py, profiles/r4zk_ring_probe.jsonl): 1500-B frames filling
// 1520-B slots want the whole-span form 0 (0.2153 ms against 0.2220 in form 2 with runs of 16), the
// 40 / 576 / 1500-B ring wants live pieces in runs of 32 (0.0919 against 0.1041 with 16), and 1500-B
// frames in 2-KiB slots live pieces in runs of 8. A launch with A.plan_out set has one extra block,
// block 0, which samples kPlanSamples datagrams evenly over the batch (the IP version and length from
// each one's first 12 bytes), while the other blocks run the batch in the form the host chose, and
// stores the plan for the NEXT batch on the same ring into coherent host memory: form 0 with the
// host's whole-span run when the layout allows it (gaps <= 64 B) and the sampled datagrams stream
// >= 7/8 of their slots; else the live pieces, in runs of about kPlanLiveBytes of STREAMED datagram
// bytes (a datagram summed inside its header window streams nothing): 8, 16 or 32 datagrams, at
// most the reach's and the batch's limit. The sampling costs the batch nothing measurable (one block
// among thousands); choosing the form inside every wave instead (each sampling 64 datagrams before
// its run) cost 3.7-10 % — an extra dependent memory round trip per wave under a saturated stream —
// and persistent waves 20 % (profiles/r5c_plan_experiments.jsonl).
constexpr uint32_t kPlanLiveBytes = 10240u;
constexpr uint32_t kPlanSamples = 1024u;

// Offset/length rings (tools/ring_probe.py RING_VARIANTS=offlengrid, profiles/r5g_ring_probe_grid.jsonl:
// runs of 8 / 16 / 32 at 5-8 waves per SIMD): short streamed datagrams (the 40 / 576 / 1500-B ring,
// mean 317 B streamed) want runs of 32 at full residency (Rx 0.1063 ms; runs of 16: 0.1267), long ones
// (1500-B frames, packed, in 1520-B or 2-KiB slots) runs of 16 at 6 waves per SIMD (2-KiB slots
// 0.2581 against 0.2696 at 8 waves; template slots 0.2290, packed 0.2251): a stream of whole 1-KiB
// pieces loses to DRAM contention at full residency, as C2 does (§5.2). Strided live runs keep full
// residency (their best at 7-8 waves on every layout) and the run rule below.
__device__ __forceinline__ void pkt_plan_vl(uint32_t mean, uint32_t& run, uint32_t& waves) {
    run = mean * 45u < kPlanLiveBytes * 2u ? 32u : 16u;
    waves = run == 32u ? 0u : 6u;
}

template <int VER, bool VL>
__device__ void pkt_plan_block(const PktBatchArgs& A) {
    __shared__ uint32_t part[4][3];
    const uint32_t m = min(A.n, kPlanSamples);
    uint32_t acc = 0u, pit = 0u, npit = 0u;
    for (uint32_t j = threadIdx.x; j < m; j += 256u) {
        const uint64_t i = ((uint64_t)j * A.n) / m;
        uintptr_t a;
        uint32_t avail;
        if constexpr (VL) {                                   // the descriptors: start, length, pitch
            const uint64_t o = A.off[i];
            a = (uintptr_t)A.base + o;
            avail = A.len[i];
            if (i + 1u < A.n) {
                const uint64_t o1 = A.off[i + 1u];
                if (o1 >= o + avail && o1 - o < 65536u) {     // in order, no overlap, near: a pitch
                    pit += (uint32_t)(o1 - o);
                    npit += 1u;
                }
            }
            if (avail < 12u) {                                 // (too short to hold a length: none)
                continue;
            }
        } else {
            a = (uintptr_t)A.base + i * A.stride;
            avail = A.len_u;
        }
        const uint32_t* p = reinterpret_cast<const uint32_t*>(a & ~(uintptr_t)3);
        const uint32_t d0 = p[0], d1 = p[1], d2 = p[2];      // the datagram's first 12 bytes (>= 64 present)
        const uint32_t sh = (uint32_t)(a & 3u);
        const uint32_t w0 = __builtin_amdgcn_alignbyte(d1, d0, sh);    // bytes 0..3
        const uint32_t w1 = __builtin_amdgcn_alignbyte(d2, d1, sh);    // bytes 4..7
        const uint32_t l4 = ((w0 >> 8) & 0xFF00u) | (w0 >> 24);          // IPv4 total length (bytes 2, 3)
        const uint32_t l6 = (((w1 & 0xFFu) << 8) | ((w1 >> 8) & 0xFFu)) + 40u;   // IPv6 payload length + 40
        const uint32_t ver = (w0 >> 4) & 0xFu;
        uint32_t L = VER == 4 ? l4 : VER == 6 ? l6 : (ver == 4u ? l4 : ver == 6u ? l6 : 0u);
        L = min(L, avail);
        acc += ((uint32_t)(a & 15u) + L <= 96u) ? 0u : L;                 // in-window datagrams stream nothing
    }
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) {
        acc += (uint32_t)__shfl_xor((int)acc, d, 64);
        pit += (uint32_t)__shfl_xor((int)pit, d, 64);
        npit += (uint32_t)__shfl_xor((int)npit, d, 64);
    }
    if ((threadIdx.x & 63u) == 0u) {
        part[threadIdx.x >> 6][0] = acc;
        part[threadIdx.x >> 6][1] = pit;
        part[threadIdx.x >> 6][2] = npit;
    }
    __syncthreads();
    if (threadIdx.x == 0u) {
        const uint32_t tot = part[0][0] + part[1][0] + part[2][0] + part[3][0];
        const uint32_t run0 = A.plan & 0xFFu;
        uint32_t cap = max((A.plan >> 8) & 0xFFu, 1u);
        uint32_t plan;
        const uint32_t mean = max(tot / max(m, 1u), 64u);
        if (!VL && run0 != 0u && (uint64_t)tot * 8u >= 7ull * m * A.stride) {
            plan = run0 << 8;                                                // form 0
        } else {
            if (VL) {                                         // a run within the reach by the sampled pitch
                const uint32_t pn = part[0][2] + part[1][2] + part[2][2] + part[3][2];
                const uint64_t pt = (uint64_t)part[0][1] + part[1][1] + part[2][1] + part[3][1];
                if (pn != 0u) {
                    cap = min(cap, max((kLiveReach - 8192u) / max((uint32_t)(pt / pn), 1u), 1u));
                }
            }
            // runs of 8, 16 or 32: the nearest on a log scale of kPlanLiveBytes / mean (offset/length:
            // pkt_plan_vl)
            uint32_t run = mean * 45u < kPlanLiveBytes * 2u ? 32u : mean * 45u < kPlanLiveBytes * 4u ? 16u : 8u;
            uint32_t waves = 0u;
            if (VL) {
                pkt_plan_vl(mean, run, waves);
            }
            plan = 2u | (min(run, cap) << 8) | (waves << 4);
            if (VL) {                                         // out of order somewhere: a wide deferred pass
                const uint32_t pn = part[0][2] + part[1][2] + part[2][2] + part[3][2];
                const uint32_t pairs = m - (A.n <= m ? 1u : 0u);
                plan |= (pn + pairs / 64u < pairs) ? 8u : 0u;
            }
        }
        // valid bit, the host's tag for this ring (a slot reused for another ring is told apart)
        const uint32_t word = 0x80000000u | (((A.plan >> 16) & 0x7FFFu) << 16) | plan;
        __hip_atomic_store(A.plan_out, word, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

// The same sampler as a launch of its own (one block), ahead of a ring's FIRST batch when the host
// waits for the plan instead of letting the first batch run unplanned (launch_pkt_plan, abi ring_plan).
template <int VER, bool VL>
__global__ void __launch_bounds__(256) pkt_plan_kernel(PktBatchArgs A) {
    pkt_plan_block<VER, VL>(A);
}

// DEF (offset/length): runs not in order within the reach are listed for the deferred pass (true) or
// done inline, one datagram at a time (false: the kernel then carries that loop, 79-93 VGPRs, 5-6 waves
// per SIMD — the residency the dense offset/length rings want anyway, so their ring plan takes this
// form and no deferred pass; profiles/r5g_ring_probe_grid.jsonl).
template <int D, bool NT, bool TX, bool REC, int VER, int BND, bool VL, bool DEF = VL>
__global__ void __launch_bounds__(256) pkt_stream_kernel(PktBatchArgs A, uint32_t spw, PktTxRecord* rec) {
    const uint32_t w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    uint32_t bid = blockIdx.x, nblk = gridDim.x;
    if (A.plan_out != nullptr) {                              // block 0: the next batch's plan
        if (bid == 0u) {
            pkt_plan_block<VER, VL>(A);
            return;
        }
        bid -= 1u;
        nblk -= 1u;
    }
    const uint32_t blk = A.xcd ? xcd_block(bid, nblk) : bid;
    pkt_stream_run<D, NT, TX, REC, VER, BND, VL, DEF>(A, spw, rec, (uint64_t)blk * 4u + w, w, threadIdx.x & 63u);
}

// Second pass of the two-pass Tx: one thread per packet writes its fields (and flags) from its record.
// WT (NETCSUM_TUNE_TX_FLUSH 1): the field bytes are stored at system scope, i.e. written through the
// L2 to HBM during this pass instead of sitting dirty in the L2 until a later launch evicts them.
// WB (TX_FLUSH 2): every wave ends with an agent-scope release (the L2 write-back of its XCD).
// WALK (IPv6 / mixed rings): the wave then finishes its datagrams whose record says EXT_HDR (chains
// past pass 1's window) with its four 16-lane groups (walk_wave, after its own field stores), so
// two-pass Tx needs no walk launch and no deferral word either.
template <bool WT, bool WB, bool WALK>
__global__ void __launch_bounds__(256) pkt_scatter_kernel(PktBatchArgs A, const PktTxRecord* rec) {
    const uint32_t i = blockIdx.x * 256u + threadIdx.x;
    bool need = false;
    if (i < A.n) {
        const uint64_t r = reinterpret_cast<const uint64_t*>(rec)[i];      // PktTxRecord, one 8-B load
        const uint32_t vals = (uint32_t)r, l4_off = (uint32_t)(r >> 32) & 0xFFFFu;
        const uint32_t flags = (uint32_t)(r >> 48) & 0xFFu, store = (uint32_t)(r >> 56);
        need = WALK && A.defer_word == nullptr && (flags & NETCSUM_PKT_EXT_HDR) != 0u;   // walk_one writes
        if (A.flags_out && !need) {                                                     // its verdict
            A.flags_out[i] = (uint8_t)flags;
        }
        if (A.fieldpos_out && !need) {
            A.fieldpos_out[i] = ((store & 1u) ? kFieldIP : 0u) | ((store & 2u) ? kFieldL4 | l4_off : 0u);
        }
        uint8_t* p = const_cast<uint8_t*>(A.base) + (A.off ? A.off[i] : (uint64_t)i * A.stride);
        if constexpr (WT) {
            if (store & 1u) {
                __hip_atomic_store(p + 10, (uint8_t)(vals & 0xFFu), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                __hip_atomic_store(p + 11, (uint8_t)((vals >> 8) & 0xFFu), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            }
            if (store & 2u) {
                __hip_atomic_store(p + l4_off, (uint8_t)((vals >> 16) & 0xFFu), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                __hip_atomic_store(p + l4_off + 1u, (uint8_t)(vals >> 24), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            }
        } else {
            if (store & 1u) {
                store_field(p + 10, vals & 0xFFFFu);
            }
            if (store & 2u) {
                store_field(p + l4_off, vals >> 16);
            }
        }
    }
    if constexpr (WALK) {
        if (A.defer_word == nullptr) {                                  // uniform
            v6walk::walk_wave<true>(A, blockIdx.x * 256u + (threadIdx.x & ~63u), need, threadIdx.x & 63u);
        }
    }
    if constexpr (WB) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");    // the wave ends when its write-back has
    }
}

// Host-memory Tx forms (netcsum_abi.hip pkt_host): one 8-B record per packet of the checksum fields
// the Tx kernels wrote into the device copy (fieldpos_out), so that only 8 B per packet return over
// PCIe instead of the chunk's bytes; the host writes the fields into its own buffer.
__global__ void __launch_bounds__(256) pkt_field_gather_kernel(PktBatchArgs A, uint64_t* rec) {
    const uint64_t i = (uint64_t)blockIdx.x * 256u + threadIdx.x;
    if (i >= A.n) {
        return;
    }
    const uint32_t pos = A.fieldpos_out[i];
    const uint8_t* p = A.base + (A.off ? A.off[i] : i * A.stride);
    uint32_t v = 0u;
    if (pos & kFieldIP) {
        v |= (uint32_t)p[10] | ((uint32_t)p[11] << 8);
    }
    if (pos & kFieldL4) {
        const uint32_t o = pos & 0xFFFFu;
        v |= ((uint32_t)p[o] | ((uint32_t)p[o + 1u] << 8)) << 16;
    }
    rec[i] = (uint64_t)v | ((uint64_t)pos << 32);
}

// TX_FLUSH 3 / 4: a separate launch of 8 / 256 one-wave workgroups, each an agent-scope release,
// after the Tx launch(es): the dirty field lines are written back before the next launch's reads.
__global__ void __launch_bounds__(64) l2_writeback_kernel() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// Completion of a zero-copy host burst (netcsum_abi.hip rx_burst_zero_copy): ONE wave, so the
// system-scope release of the completion store waits for every result store before it (vmcnt is
// per wave). Results are copied as whole 16-B chunks (the device buffers hold whole chunks).
__global__ void __launch_bounds__(64) burst_done_kernel(const uint8_t* fl, const uint8_t* act, uint32_t n,
                                                        uint8_t* h_fl, uint8_t* h_act, unsigned long long* word,
                                                        uint32_t tag) {
    const uint32_t chunks = (n + 15u) >> 4;
    for (uint32_t c = threadIdx.x; c < chunks; c += 64u) {
        reinterpret_cast<u32x4*>(h_fl)[c] = reinterpret_cast<const u32x4*>(fl)[c];
        if (act != nullptr) {
            reinterpret_cast<u32x4*>(h_act)[c] = reinterpret_cast<const u32x4*>(act)[c];
        }
    }
    if (threadIdx.x == 0u) {
        __hip_atomic_store(word, (unsigned long long)tag, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

// ---- resident burst server (NETCSUM_TUNE_BURST_ZERO_COPY 3; netcsum_abi.hip burst_server_post)
// A small burst's work is a few PCIe round trips; a kernel launch per burst costs more than that. The
// server is launched once and stays: wave 0 of each block (the leader) polls the post line, a 64-B
// line of coherent host memory read as a whole (one request: its check catches a read that tore it),
// and hands a burst it has not served to its block through LDS; the block's 4 waves then take runs
// blockIdx * 4 + w, + 4 * blocks, ... of the burst with the run-stream code above (mixed IPv4 / IPv6,
// 4 pieces in flight), write the results into coherent host memory and release them. A block stops
// when it has been idle for idle_ticks, when life_ticks have passed since it started (even while
// bursts keep coming: the server's stream shares a hardware queue with other streams of the process,
// GPU_MAX_HW_QUEUES, and their kernels wait behind it), or when it sees another block's closed mark
// (the marks are read with the post line, so the blocks stop together and the host, which waits for
// the whole grid, waits for one burst at most). Stopping is Dekker's handshake with the host: the
// block marks itself closed, fences, and reads the line once more; the host posts, fences and reads
// the marks, so a burst posted meanwhile is taken here or found by the host, which waits the server
// out and relaunches it when the burst is unserved.
constexpr uint32_t kServeRun = 1u, kServeExit = 2u;

__device__ uint32_t burst_leader_wait(const BurstServerArgs& S, uint64_t seen, uint64_t t_start, uint32_t lane,
                                      uint32_t* s_line) {
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    const uint32_t nb = gridDim.x;
    bool closing = false;
    for (;;) {
        uint64_t v = 0u;
        if (lane < 8u) {                                        // lanes 0..7: the line's 8 quadwords
            v = __hip_atomic_load(reinterpret_cast<const uint64_t*>(S.post) + lane, __ATOMIC_RELAXED,
                                  __HIP_MEMORY_SCOPE_SYSTEM);
        } else if (lane < 8u + nb) {                            // lanes 8..: every block's closed mark
            v = __hip_atomic_load(S.closed + (lane - 8u), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        }
        const bool others_closed = __ballot(lane >= 8u && lane < 8u + nb && v != 0u) != 0u;
        uint32_t d[12];
#pragma unroll
        for (int i = 0; i < 6; ++i) {
            d[2 * i] = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, i);
            d[2 * i + 1] = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(v >> 32), i);
        }
        BurstPost p{};
        p.seq = ((uint64_t)d[1] << 32) | d[0];
        p.ring = ((uint64_t)d[3] << 32) | d[2];
        p.stride = d[4];
        p.n = d[5];
        p.pkt_len = d[6];
        p.spw = d[7];
        p.form = d[8];
        p.udp_mode = d[9];
        p.rx_cfg = d[10];
        p.check = d[11];
        if (p.seq != seen && p.check == burst_post_check(p)) {
            if (lane < 6u) {
                s_line[2u * lane] = (uint32_t)v;
                s_line[2u * lane + 1u] = (uint32_t)(v >> 32);
            }
            return p.seq == kBurstStop ? kServeExit
                   : (closing || others_closed) ? (kServeRun | kServeExit) : kServeRun;
        }
        if (closing) {
            return kServeExit;
        }
        const uint64_t now = __builtin_amdgcn_s_memrealtime();
        if (others_closed || now - t0 > S.idle_ticks || now - t_start > S.life_ticks) {
            closing = true;
            if (lane == 0u) {
                __hip_atomic_store(S.closed + blockIdx.x, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            }
            __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "");       // the mark before the line's last read
            continue;
        }
        __builtin_amdgcn_s_sleep(2);
    }
}

template <bool TX, int BND, bool VL>
__device__ __forceinline__ void burst_serve(const PktBatchArgs& A, uint32_t spw, PktTxRecord* rec, uint32_t w,
                                            uint32_t lane) {
    const uint32_t runs = (A.n + spw - 1u) / spw;
    for (uint32_t r = blockIdx.x * 4u + w; r < runs; r += gridDim.x * 4u) {
        pkt_stream_run<4, true, TX, TX, 0, BND, VL>(A, spw, rec, r, w, lane);
    }
}

__global__ void __launch_bounds__(256) burst_server_kernel(BurstServerArgs S) {
    __shared__ uint32_t s_line[12];
    __shared__ uint32_t s_cmd;
    const uint32_t w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint32_t lane = threadIdx.x & 63u;
    const uint64_t t_start = __builtin_amdgcn_s_memrealtime();
    uint64_t seen = S.seq0;
    for (;;) {
        if (w == 0u) {
            const uint32_t cmd = burst_leader_wait(S, seen, t_start, lane, s_line);
            if (lane == 0u) {
                s_cmd = cmd;
            }
        }
        __syncthreads();
        const uint32_t cmd = __builtin_amdgcn_readfirstlane(s_cmd);
        if (cmd & kServeRun) {
            uint32_t d[12];
#pragma unroll
            for (int i = 0; i < 12; ++i) {
                d[i] = __builtin_amdgcn_readfirstlane(s_line[i]);
            }
            PktBatchArgs A{};
            A.base = reinterpret_cast<const uint8_t*>(((uint64_t)d[3] << 32) | d[2]);
            A.stride = d[4];
            A.n = d[5];
            A.len_u = d[6];
            const uint32_t spw = d[7], form = d[8];
            A.udp_tx_csum = d[9];
            A.rx_cfg = d[10];
            if ((form >> 1) == kBurstOffLen) {
                A.off = S.off;
                A.len = S.len;
            }
            // a wave with runs of this burst: the ring's and descriptors' bytes fresh from host memory
            // (L1 / L2 invalidate)
            if (blockIdx.x * 4u + w < (A.n + spw - 1u) / spw) {
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
            }
            if (form & 1u) {
                if ((form >> 1) == kBurstWhole) {
                    burst_serve<true, 0, false>(A, spw, S.rec, w, lane);
                } else if ((form >> 1) == kBurstLive) {
                    burst_serve<true, 2, false>(A, spw, S.rec, w, lane);
                } else {
                    burst_serve<true, 2, true>(A, spw, S.rec, w, lane);
                }
            } else {
                A.flags_out = S.flags;
                A.action_out = S.act;
                if ((form >> 1) == kBurstWhole) {
                    burst_serve<false, 0, false>(A, spw, nullptr, w, lane);
                } else if ((form >> 1) == kBurstLive) {
                    burst_serve<false, 2, false>(A, spw, nullptr, w, lane);
                } else {
                    burst_serve<false, 2, true>(A, spw, nullptr, w, lane);
                }
            }
            seen = ((uint64_t)d[1] << 32) | d[0];
            // the block's result stores have reached the L2 (the barrier's release), then one
            // system-scope release writes them back to host memory. (Per wave: 64 frames 12.5 us;
            // system-scope loads and stores instead of fences 13.0 us for Tx and 23.8 us for Rx, whose
            // byte stores then cross PCIe one by one: tools/burst_latency.c zc, profiles/r4p_burst_zc.jsonl)
            __syncthreads();
            if (w == 0u && blockIdx.x * 4u < (A.n + spw - 1u) / spw) {
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
            }
        }
        if (cmd & kServeExit) {
            break;
        }
        __syncthreads();                                        // s_line / s_cmd free for the next post
    }
}

thread_local TuneKnob g_tx_flush{-1};

int tx_flush_mode() {
    const int m = g_tx_flush.load(std::memory_order_relaxed);
    return m < 0 ? 0 : m;
}

template <bool WALK>
hipError_t launch_scatter(const PktBatchArgs& a, const PktTxRecord* rec, hipStream_t s) {
    const int m = tx_flush_mode();
    const dim3 g((a.n + 255u) / 256u), b(256);
    if (m == 1) {
        hipLaunchKernelGGL((pkt_scatter_kernel<true, false, WALK>), g, b, 0, s, a, rec);
    } else if (m == 2) {
        hipLaunchKernelGGL((pkt_scatter_kernel<false, true, WALK>), g, b, 0, s, a, rec);
    } else {
        hipLaunchKernelGGL((pkt_scatter_kernel<false, false, WALK>), g, b, 0, s, a, rec);
    }
    return hipGetLastError();
}

hipError_t launch_tx_flush(hipStream_t s) {
    const int m = tx_flush_mode();
    if (m == 3 || m == 4) {
        hipLaunchKernelGGL(l2_writeback_kernel, dim3(m == 3 ? 8 : 256), dim3(64), 0, s);
        return hipGetLastError();
    }
    return hipSuccess;
}

thread_local bool tls_fault_skip_deferred = false;

// the deferred pass, unless a test asked for its launch to fail (set_fault_skip_deferred)
template <int D, bool NT, bool TX, bool REC, int VER, int BND>
hipError_t launch_vl_deferred(const PktBatchArgs& a, int dgrid, uint32_t spw, PktTxRecord* rec, hipStream_t s) {
    if (tls_fault_skip_deferred) {
        tls_fault_skip_deferred = false;
        return hipErrorLaunchFailure;
    }
    hipLaunchKernelGGL((pkt_vl_deferred_kernel<D, NT, TX, REC, VER, BND>), dim3(dgrid), dim3(256), 0, s, a, spw, rec);
    return hipGetLastError();
}

template <int D, bool NT, bool TX, int VER, int BND, bool VL>
hipError_t launch_pkt_stream_t(const PktBatchArgs& a0, uint32_t spw, hipStream_t s, PktTxRecord* rec, bool scatter) {
    PktBatchArgs a = a0;
    // no piece touch by default: the header prologue already loads each packet's first bytes with
    // the plain policy, and touching every piece on top is slower (r2ct: Rx 0.2174 -> 0.2315 ms)
    a.touch = stream_touch(false) ? 1u : 0u;
    a.xcd = stream_xcd(false) ? 1u : 0u;
    const uint64_t waves = ((uint64_t)a.n + spw - 1u) / spw;
    const int grid = (int)((waves + 3u) / 4u) + (a.plan_out != nullptr ? 1 : 0);   // (+ the plan block)
    const uint32_t lds = stream_lds_bytes((int)a.res_waves);
    // offset/length: the deferred pass (8 blocks for a ring in order, else up to one per CU: a batch
    // whose every run is listed is slow, but correct)
    const int dgrid = a.vl_wide ? (int)std::min<uint64_t>((waves + 3u) / 4u, 2048u) : (int)std::min<uint64_t>((waves + 3u) / 4u, 8u);
    if (TX && rec != nullptr) {
        if (VL && a.vl_ctr == nullptr) {                      // (offset/length, inline: no deferred pass)
            hipLaunchKernelGGL((pkt_stream_kernel<D, NT, TX, TX, VER, BND, VL, false>), dim3(grid), dim3(256), lds, s, a, spw, rec);
        } else {
            hipLaunchKernelGGL((pkt_stream_kernel<D, NT, TX, TX, VER, BND, VL>), dim3(grid), dim3(256), lds, s, a, spw, rec);
        }
        hipError_t e = hipGetLastError();
        if (e == hipSuccess && VL && a.vl_ctr != nullptr) {
            if constexpr (VL) {
                e = launch_vl_deferred<D, NT, TX, TX, VER, BND>(a, dgrid, spw, rec, s);
            }
        }
        if (e != hipSuccess || !scatter) return e;
        e = launch_scatter<VER != 4>(a, rec, s);
        return e != hipSuccess ? e : launch_tx_flush(s);
    }
    if (VL && a.vl_ctr == nullptr) {
        hipLaunchKernelGGL((pkt_stream_kernel<D, NT, TX, false, VER, BND, VL, false>), dim3(grid), dim3(256), lds, s, a, spw, rec);
    } else {
        hipLaunchKernelGGL((pkt_stream_kernel<D, NT, TX, false, VER, BND, VL>), dim3(grid), dim3(256), lds, s, a, spw, rec);
    }
    hipError_t e = hipGetLastError();
    if (e == hipSuccess && VL && a.vl_ctr != nullptr) {
        if constexpr (VL) {
            e = launch_vl_deferred<D, NT, TX, false, VER, BND>(a, dgrid, spw, rec, s);
        }
    }
    return (e != hipSuccess || !TX) ? e : launch_tx_flush(s);
}

}  // namespace

void set_fault_skip_deferred(bool on) {
    tls_fault_skip_deferred = on;
}

hipError_t launch_pkt_field_gather(const PktBatchArgs& a, uint64_t* rec_out, hipStream_t s) {
    if (a.n == 0u) return hipSuccess;
    if (a.fieldpos_out == nullptr || rec_out == nullptr) return hipErrorInvalidValue;
    hipLaunchKernelGGL(pkt_field_gather_kernel, dim3((unsigned)(((uint64_t)a.n + 255u) / 256u)), dim3(256), 0, s, a, rec_out);
    return hipGetLastError();
}

hipError_t launch_burst_done(const uint8_t* fl, const uint8_t* act, uint32_t n, uint8_t* h_fl, uint8_t* h_act,
                             unsigned long long* word, uint32_t tag, hipStream_t s) {
    hipLaunchKernelGGL(burst_done_kernel, dim3(1), dim3(64), 0, s, fl, act, n, h_fl, h_act, word, tag);
    return hipGetLastError();
}

hipError_t launch_burst_server(const BurstServerArgs& a, int blocks, hipStream_t s) {
    if (blocks < 1 || blocks > kBurstServerMaxBlocks || a.post == nullptr || a.closed == nullptr) {
        return hipErrorInvalidValue;
    }
    hipLaunchKernelGGL(burst_server_kernel, dim3(blocks), dim3(256), 0, s, a);
    return hipGetLastError();
}

void set_tx_flush(int mode) {
    g_tx_flush.store(mode);
}

// Strided batches of >= 64-B packets (IPv4, IPv6 or mixed) whose runs span < 2^31 bytes: any gap
// between slots in the live-piece forms of bounds 1 and 2, at most 64 B in the others (bound 0, and
// bound 3, which loads a run's first pieces whole); offset/length batches in bounds 1 and 2.
bool pkt_stream_supported(const PktBatchArgs& a, int ip_ver, int bound) {
    if (!(ip_ver == 4 || ip_ver == 6 || ip_ver == 0)) return false;
    if (a.off != nullptr) return (bound == 1 || bound == 2) && a.len != nullptr;
    if (bound >= 1 && a.len_u + 128u > kLiveReach) return false;        // a run of one spans <= 63 KiB
    return a.len_u >= 64u && a.stride >= a.len_u && ((bound == 1 || bound == 2) || a.stride <= a.len_u + 64u) &&
           (uint64_t)kMaxRunPkts * a.stride < (1ull << 31);
}

hipError_t launch_pkt_plan(const PktBatchArgs& a, int ip_ver, hipStream_t s) {
    if (a.plan_out == nullptr || a.n == 0u) return hipErrorInvalidValue;
    const bool vl = a.off != nullptr;
#define NETCSUM_PP(V_, VL_) \
    if (ip_ver == V_ && vl == VL_) { hipLaunchKernelGGL((pkt_plan_kernel<V_, VL_>), dim3(1), dim3(256), 0, s, a); return hipGetLastError(); }
    NETCSUM_PP(4, false) NETCSUM_PP(4, true) NETCSUM_PP(6, false) NETCSUM_PP(6, true) NETCSUM_PP(0, false) NETCSUM_PP(0, true)
#undef NETCSUM_PP
    return hipErrorInvalidValue;
}

hipError_t launch_pkt_stream(const PktBatchArgs& a, int ip_ver, int depth, uint32_t spw, bool nt, bool tx, int bound,
                             hipStream_t s, PktTxRecord* rec, bool scatter) {
    if (spw == 0u || spw > kMaxRunPkts || bound < 0 || bound > 3 || !pkt_stream_supported(a, ip_ver, bound)) {
        return hipErrorInvalidValue;
    }
    // live pieces: a strided run spans at most 64 pieces (the host sizes runs for it; offset/length
    // runs check their span on the device)
    if (bound >= 1 && a.off == nullptr && 128u + (uint64_t)(spw - 1u) * a.stride + a.len_u > kLiveReach) {
        return hipErrorInvalidValue;
    }
    // the plan block: its candidate runs must be legal for this layout (the next batch runs them)
    if (a.res_waves > 8u) {
        return hipErrorInvalidValue;
    }
    if (a.plan_out != nullptr && a.off == nullptr) {
        const uint32_t run0 = a.plan & 0xFFu, cap = (a.plan >> 8) & 0xFFu;
        if (cap == 0u || cap > kMaxRunPkts || run0 > kMaxRunPkts || 128u + (uint64_t)(cap - 1u) * a.stride + a.len_u > kLiveReach ||
            (run0 != 0u && !pkt_stream_supported(a, ip_ver, 0))) {
            return hipErrorInvalidValue;
        }
    }
    const bool vl = a.off != nullptr;
    // every bound with 4 pieces in flight, 8 with bounds 0, 2 and 3; offset/length runs in the
    // live-piece forms 1 and 2
#define NETCSUM_P(V_, D_, NT_, TX_, B_, VL_)                                                              \
    if (ip_ver == V_ && depth == D_ && nt == NT_ && tx == TX_ && bound == B_ && vl == VL_)                 \
        return launch_pkt_stream_t<D_, NT_, TX_, V_, B_, VL_>(a, spw, s, rec, scatter);
#define NETCSUM_PB(V_, D_, B_, VL_)                                                                       \
    NETCSUM_P(V_, D_, true, false, B_, VL_) NETCSUM_P(V_, D_, false, false, B_, VL_)                      \
    NETCSUM_P(V_, D_, true, true, B_, VL_) NETCSUM_P(V_, D_, false, true, B_, VL_)
#define NETCSUM_PV(V_) NETCSUM_PB(V_, 4, 0, false) NETCSUM_PB(V_, 4, 1, false) NETCSUM_PB(V_, 4, 2, false)     \
    NETCSUM_PB(V_, 4, 3, false) NETCSUM_PB(V_, 8, 0, false) NETCSUM_PB(V_, 8, 2, false) NETCSUM_PB(V_, 8, 3, false) \
    NETCSUM_PB(V_, 4, 1, true) NETCSUM_PB(V_, 4, 2, true) NETCSUM_PB(V_, 8, 2, true)
    NETCSUM_PV(4) NETCSUM_PV(6) NETCSUM_PV(0)
#undef NETCSUM_PV
#undef NETCSUM_PB
#undef NETCSUM_P
    return hipErrorInvalidValue;
}

}  // namespace netcsum
