// netcsum_v6walk.hip — IPv6 extension-header chains of any length in the packet batches.
//
// The batch kernels (netcsum_packets.hip, netcsum_pktstream.hip) parse each datagram from the bytes
// their first loads hold (a 96 - lead / 16 G - lead byte window) and walk at most 4 extension
// headers; a chain past that comes back as NETCSUM_PKT_EXT_HDR. The reference walks any chain
// (NetIPv6_RxPktProcessExtHdr, net_ipv6.c:8396-8510: Hop-by-Hop / Destination Options via
// NetIPv6_RxOptHdr, Routing via NetIPv6_RxRoutingHdr, length (HdrExtLen + 1) * 8, net_ipv6.c:8601,
// until the next header is not an extension header), so this pass finishes exactly those datagrams:
//
//   one wave per 64 flags; the datagrams whose flag has EXT_HDR are found by a ballot, and a 16-lane
//   group of the wave takes each of them (four at a time): the chain is walked with group-uniform loads (no window, no header
//   count), then the transport part [off, tot) and the addresses [8, 40) are summed with the group's
//   16 lanes reading half-words in parallel, and the verdict (Rx) or the checksum field (Tx) and the
//   flag are written by the group's lane 0 (vector stores).
//
// Datagrams are rare on this path (option headers, chains of more than 4 routing headers or longer
// than ~50 bytes), and the pass is launched only when the batch kernels deferred one (their
// deferral word, launch_pkt_v6_walk). The verdict rules are pkt_parse_v6's (netcsum_packets.hip; the same reference lines):
//   TCP (6)     DataVerify / DataCalc + pseudo {src, dst, ulen, 0, 6}        net_tcp.c:7871-7879, 29839-29862
//   UDP (17)    length check, field 0 = no checksum (Rx), 0 -> 0xFFFF (Tx)   net_udp.c:1903-1957, 2909-2937
//   ICMPv6 (58) Rx types 1, 3, 4 without the pseudo-header, 128-131 / 134-137 with it, others no verdict;
//               Tx every type with it                                         net_icmpv6.c:2910-2948, 1439
// with ulen = payload length - extension-header bytes (net_ipv6.c:5682); Fragment (44) -> FRAGMENT,
// another extension header, a late Hop-by-Hop, an option with a discard action or a routing type > 2
// with Segments Left != 0 -> EXT_HDR (no transport verdict: the reference drops those,
// net_ipv6.c:8307-8309, 8465-8476, 8630-8671, 8735-8753), a header running past the payload ->
// MALFORMED. The batch kernels leave every datagram with a Hop-by-Hop or Destination Options header
// to this pass (its options must be walked).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "netcsum_device.h"
#include "netcsum_kernels.h"
#include "netcsum_v6walk.h"

namespace netcsum {

namespace {

// One flag per lane, one wave per 64 datagrams: a batch in which every datagram needs the walk (an
// adversarial ring of long chains) spreads over n / 64 waves instead of queueing behind a few (a
// 16-flags-per-lane scan read the flags no faster: 4.8 us per 1 M either way, profiles/r2zt_*), and
// the wave's four 16-lane groups take the next four flagged datagrams at a time (their dependent
// chain loads overlap).
template <bool TX>
__global__ void __launch_bounds__(256) pkt_v6_walk_kernel(PktBatchArgs A) {
    if (A.defer_word != nullptr && *A.defer_word != A.defer_tag) {
        return;                                     // no batch kernel deferred a datagram this call
    }
    const uint32_t lane = threadIdx.x & 63u;
    for (uint64_t w0 = (uint64_t)blockIdx.x * 256u + (threadIdx.x & ~63u); w0 < A.n; w0 += (uint64_t)gridDim.x * 256u) {
        const uint64_t i = w0 + lane;
        const bool need = i < A.n && (A.flags_out[i] & v6walk::W_EXT_HDR) != 0u;
        v6walk::walk_wave<TX>(A, (uint32_t)w0, need, lane);
    }
}

}  // namespace

hipError_t launch_pkt_v6_walk(const PktBatchArgs& a, bool tx, int cus, hipStream_t s) {
    if (a.n == 0u) return hipSuccess;
    if (a.flags_out == nullptr) return hipErrorInvalidValue;
    const uint64_t blocks = ((uint64_t)a.n + 255u) / 256u;
    const int grid = (int)std::min<uint64_t>(blocks, (uint64_t)std::max(cus, 1) * 64u);
    if (tx) {
        hipLaunchKernelGGL(pkt_v6_walk_kernel<true>, dim3(grid), dim3(256), 0, s, a);
    } else {
        hipLaunchKernelGGL(pkt_v6_walk_kernel<false>, dim3(grid), dim3(256), 0, s, a);
    }
    return hipGetLastError();
}

}  // namespace netcsum
