/*
 * netcsum_burst.c — host side of the checksum-offload burst adapters (include/netcsum_mi355x.h
 * (2b'')). Plain C11, host logic only.
 *
 * NetUtil_MI355X_RxBurstTally turns a burst's per-frame actions into the error-counter increments
 * the reference's stack would have made at its checksum checks (NET_CTR_ERR_INC at
 * net_ipv4.c:5252, net_tcp.c:7887, net_udp.c:1965 / :1975, net_icmpv4.c:1698, net_igmp.c:1336,
 * net_icmpv6.c:2953), so an integration that drops frames before NetIF_Rx can still account for
 * them in Net_ErrCtrs.
 */
#include "../../include/netcsum_mi355x.h"

NET_ERR NetUtil_MI355X_RxBurstTally(const uint8_t *h_action, uint32_t n_pkt, uint32_t *ctr)
{
    uint32_t i;

    if (ctr == NULL || (h_action == NULL && n_pkt != 0u)) {
        return NET_ERR_FAULT_NULL_PTR;
    }
    for (i = 0u; i < n_pkt; ++i) {
        if (h_action[i] >= NETCSUM_RX_NBR_ACTIONS) {
            return (NET_ERR)NET_UTIL_ERR_MI355X_INVALID_ARG;
        }
    }
    for (i = 0u; i < n_pkt; ++i) {
        ctr[h_action[i]] += 1u;
    }
    return NET_UTIL_ERR_NONE;
}
