/*
 * netcsum_shard.c — multi-GPU partitioning of a batch. Plain C11, host logic only.
 *
 * Segments are independent (one checksum each, net_util.c:344-449 per segment), so a batch shards
 * into contiguous index ranges with no exchange step. A uniform batch (C2 / C5) splits by count;
 * a variable-length batch (C4: UDP datagrams of 40-9000 B) splits by BYTES — a prefix sum of
 * len_i + pseudo_len over the batch, rank r taking the segments whose prefix falls in
 * [r*T/world, (r+1)*T/world) — so every GPU streams the same HBM bytes to within one segment.
 */
#include "../../include/netcsum_mi355x.h"

NET_ERR NetUtil_MI355X_ShardVarLen(const uint16_t *seg_len, uint32_t n_seg, CPU_INT16U pseudo_len,
                                   uint32_t world, uint32_t *first)
{
    uint64_t total = 0u, acc = 0u;
    uint32_t i, r = 1u;

    if (first == NULL || (seg_len == NULL && n_seg != 0u)) {
        return NET_ERR_FAULT_NULL_PTR;
    }
    if (world == 0u) {
        return (NET_ERR)NET_UTIL_ERR_MI355X_INVALID_ARG;
    }
    for (i = 0u; i < n_seg; ++i) {
        total += (uint64_t)seg_len[i] + pseudo_len;
    }
    first[0] = 0u;
    /* rank r starts at the first segment whose start offset acc satisfies acc >= r*T/world, i.e.
     * acc*world >= r*T (exact in u64 for any batch < 2^32 segments of < 2^17 B, world < 2^15), so
     * each boundary is off by less than one segment */
    for (i = 0u; i < n_seg && r < world; ++i) {
        while (r < world && acc * world >= (uint64_t)r * total) {
            first[r++] = i;
        }
        acc += (uint64_t)seg_len[i] + pseudo_len;
    }
    while (r < world) {
        first[r++] = n_seg;
    }
    first[world] = n_seg;
    return NET_UTIL_ERR_NONE;
}
