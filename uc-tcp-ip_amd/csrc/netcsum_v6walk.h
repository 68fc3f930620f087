// netcsum_v6walk.h — the IPv6 extension-header walk of one datagram by a 16-lane group (walk_one),
// shared by the walk pass (netcsum_v6walk.hip, after the Tx and lane-group batch kernels) and by the
// run-stream Rx kernel (netcsum_pktstream.hip), which finishes its own deferred datagrams at the end
// of each run. See netcsum_v6walk.hip for the rules and the reference lines they follow.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "netcsum_device.h"
#include "netcsum_kernels.h"

namespace netcsum {
namespace v6walk {

constexpr uint32_t W_IP_OK = 0x01u, W_L4_OK = 0x02u, W_L4_CHECKED = 0x04u, W_UDP_NO_CSUM = 0x08u,
                   W_MALFORMED = 0x10u, W_FRAGMENT = 0x20u, W_L4_MALFORMED = 0x40u, W_EXT_HDR = 0x80u;

__device__ __forceinline__ bool ext_hdr_value(uint32_t nh) {   // net_ipv6.h NET_IP_HDR_PROTOCOL_EXT_*
    return nh == 0u || nh == 43u || nh == 44u || nh == 50u || nh == 51u || nh == 59u || nh == 60u ||
           nh == 135u || nh == 139u || nh == 140u || nh == 253u || nh == 254u;
}

__device__ __forceinline__ uint32_t be16(const uint8_t* p, uint32_t k) {
    return ((uint32_t)p[k] << 8) | (uint32_t)p[k + 1u];
}

// NetIPv6_RxOptHdr's option walk (net_ipv6.c:8604-8672) over a Hop-by-Hop / Destination Options
// header h of eh_len octets: an option whose type & 0x1F is not Pad1 (0), PadN (1) or Router Alert
// (5) and whose action bits (type & 0xC0) are not "skip" (0x00) drops the datagram
// (NET_IPv6_ERR_INVALID_EH_OPT); Pad1 advances one octet, every other option Len + 2. An option that
// starts at the header's last octet would have its Len read one past the header, but any value ends
// the walk there, so that octet is not read. Group-uniform byte loads (one cached line per 64 B).
__device__ __forceinline__ bool options_accept(const uint8_t* h, uint32_t eh_len) {
    for (uint32_t nto = 0u; nto + 2u < eh_len;) {
        const uint32_t t = h[2u + nto];
        const uint32_t opt = t & 0x1Fu;
        if (opt != 0u && opt != 1u && opt != 5u && (t & 0xC0u) != 0u) {
            return false;
        }
        nto += (opt == 0u) ? 1u : ((nto + 3u < eh_len ? (uint32_t)h[3u + nto] : 0u) + 2u);
    }
    return true;
}

// NetIPv6_RxRoutingHdr (net_ipv6.c:8735-8753): routing types 0, 1, 2 pass; any other type drops the
// datagram (NET_IPv6_ERR_INVALID_EH_OPT_SEQ) unless Segments Left is 0.
__device__ __forceinline__ bool routing_accepts(const uint8_t* h) {
    return h[2] <= 2u || h[3] == 0u;
}

// A datagram is finished by a group of kLanes lanes (a wave takes 4 datagrams at a time).
constexpr uint32_t kLanes = 16u;

// Ones'-complement sum, in big-endian half-words of the datagram, of its bytes [lo, hi) (lo even; an
// odd last octet padded with zero), the half-word at `skip` (even, or ~0u) counted as zero, folded to
// 16 bits (0 iff every counted octet is 0). The group's lanes read whole aligned 16-B chunks (bytes
// outside [lo, hi) masked; a chunk never leaves the 16-B block, hence the page, of a datagram byte)
// and add their little-endian half-words with v_sad_u16: with the datagram at an even address those
// are the big-endian ones byte-swapped, at an odd address they ARE the big-endian ones (RFC 1071 §2).
__device__ __forceinline__ uint32_t group_sum(const uint8_t* p, uint32_t lo, uint32_t hi, uint32_t skip, uint32_t lane) {
    const uintptr_t s0 = (uintptr_t)p + lo, e0 = (uintptr_t)p + hi;
    uint32_t s = 0u;
    for (uintptr_t c = (s0 & ~(uintptr_t)15u) + 16u * lane; c < e0; c += 16u * kLanes) {
        const u32x4 v = *reinterpret_cast<gu32x4*>(c);
        s = sum4(mask_chunk(v, (int)((intptr_t)s0 - (intptr_t)c), (int)((intptr_t)e0 - (intptr_t)c)), s);
    }                                               // <= 258 chunks of 8 half-words per lane
#pragma unroll
    for (int o = (int)kLanes / 2; o > 0; o >>= 1) {
        s += (uint32_t)__shfl_xor((int)s, o, (int)kLanes);
    }                                               // < 2^32: 32 788 half-words at most
    const uint32_t odd = (uint32_t)((uintptr_t)p & 1u);
    if (skip != ~0u) {                              // exact: those two octets were added above
        s -= ((uint32_t)p[skip] << (8u * odd)) + ((uint32_t)p[skip + 1u] << (8u * (odd ^ 1u)));
    }
    const uint32_t r = fold16(s);
    return odd ? r : rot8(r);
}

// A lane group finishes datagram i (all values below are uniform in the group; lane = its lane).
template <bool TX>
__device__ __forceinline__ void walk_one(const PktBatchArgs& A, uint32_t i, uint32_t lane) {
    uint64_t off64;
    uint32_t avail;
    if (A.off) {
        off64 = A.off[i];
        avail = A.len[i];
    } else {
        off64 = (uint64_t)i * A.stride;
        avail = A.len_u;
    }
    uint8_t* p = const_cast<uint8_t*>(A.base) + off64;
    if (avail < 40u || (p[0] >> 4) != 6u) {
        return;                                     // not IPv6: the batch kernel's flag stands
    }
    const uint32_t tot = 40u + be16(p, 4u);
    if (tot > avail) {
        return;                                     // MALFORMED already (never EXT_HDR)
    }
    uint32_t nh = p[6], off = 40u, f = 0u;
    while (nh == 0u || nh == 43u || nh == 60u) {   // off grows by >= 8 per header: ends by tot
        if (nh == 0u && off != 40u) {
            f = W_IP_OK | W_EXT_HDR;                // Hop-by-Hop only first (net_ipv6.c:8307)
            break;
        }
        if (off + 8u > tot) {
            f = W_MALFORMED;                        // the header would run past the payload
            break;
        }
        const uint32_t eh_len = ((uint32_t)p[off + 1u] + 1u) * 8u;
        if (off + eh_len > tot) {
            f = W_MALFORMED;                        // (the reference reads on past the payload)
            break;
        }
        if (!(nh == 43u ? routing_accepts(p + off) : options_accept(p + off, eh_len))) {
            f = W_IP_OK | W_EXT_HDR;                // the reference drops the datagram here
            break;
        }
        nh = p[off];
        off += eh_len;
    }
    uint32_t csum_off = ~0u;
    bool pseudo = false, check = false;
    if (f == 0u) {
        f = W_IP_OK;
        const uint32_t ulen = tot - off;
        if (nh == 44u) {
            f |= W_FRAGMENT;
        } else if (ext_hdr_value(nh)) {
            f |= W_EXT_HDR;
        } else if (nh == 6u) {
            if (ulen < 20u) {
                f |= W_L4_MALFORMED;
            } else {
                csum_off = off + 16u;
                pseudo = check = true;
            }
        } else if (nh == 17u) {
            if (ulen < 8u || be16(p, off + 4u) != ulen) {
                f |= W_L4_MALFORMED;
            } else {
                csum_off = off + 6u;
                if (!TX && be16(p, off + 6u) == 0u) {
                    f |= W_UDP_NO_CSUM | W_L4_OK;
                } else if (TX && !udp_tx_compute(A.udp_tx_csum, be16(p, off + 6u))) {
                    f |= W_UDP_NO_CSUM;
                    if (lane == 0u) {
                        p[csum_off] = 0u;           // NET_UDP_HDR_CHK_SUM_NONE (net_udp.c:2935)
                        p[csum_off + 1u] = 0u;
                        if (A.fieldpos_out) A.fieldpos_out[i] = kFieldL4 | csum_off;
                    }
                } else {
                    pseudo = check = true;
                }
            }
        } else if (nh == 58u) {
            if (ulen < 4u) {
                f |= W_L4_MALFORMED;
            } else {
                csum_off = off + 2u;
                const uint32_t type = p[off];
                if (TX || (type >= 128u && type <= 131u) || (type >= 134u && type <= 137u)) {
                    pseudo = check = true;
                } else if (type == 1u || type == 3u || type == 4u) {
                    check = true;                   // HdrVerify over the message alone
                }
            }
        }
    }
    if (check) {
        uint32_t s = group_sum(p, off, tot, TX ? csum_off : ~0u, lane);
        if (pseudo) {
            s += group_sum(p, 8u, 40u, ~0u, lane) + (tot - off) + nh;   // addresses, length, next header
        }                                           // (folded values: no overflow)
        const uint32_t r = fold16(s);
        if constexpr (TX) {
            uint32_t c = (~r) & 0xFFFFu;
            if (nh == 17u && c == 0u) {
                c = 0xFFFFu;                        // RFC 768 (net_udp.c:2929-2931)
            }
            if (lane == 0u) {
                p[csum_off] = (uint8_t)(c >> 8);
                p[csum_off + 1u] = (uint8_t)c;
                if (A.fieldpos_out) A.fieldpos_out[i] = kFieldL4 | csum_off;
            }
            f |= W_L4_CHECKED | W_L4_OK;
        } else {
            f |= W_L4_CHECKED | (r == 0xFFFFu ? W_L4_OK : 0u);
        }
    }
    if (lane == 0u) {
        if (A.flags_out) A.flags_out[i] = (uint8_t)f;
        if (!TX && A.action_out) {
            A.action_out[i] = (uint8_t)rx_action(f, nh, true, A.rx_cfg);
        }
    }
}


// The calling wave's datagrams s0 + k whose lane k has `need` set, four at a time by its 16-lane
// groups (every lane of the wave must be active).
template <bool TX>
__device__ __forceinline__ void walk_wave(const PktBatchArgs& A, uint32_t s0, bool need, uint32_t lane) {
    const uint32_t grp = lane / kLanes;
    uint64_t m = __ballot(need);                    // wave-uniform
    while (m != 0u) {                               // group g takes the g-th lowest set bit
        uint32_t j = ~0u;
#pragma unroll
        for (uint32_t g = 0; g < 64u / kLanes; ++g) {
            if (m != 0u) {
                j = (g == grp) ? (uint32_t)__builtin_ctzll(m) : j;
                m &= m - 1u;
            }
        }
        if (j != ~0u) {
            walk_one<TX>(A, s0 + j, lane % kLanes);
        }
    }
}

}  // namespace v6walk
}  // namespace netcsum
