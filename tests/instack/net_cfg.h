/* In-stack compile check: the stack configuration the drop-in reads (template values,
 * Cfg/Template/net_cfg.h:184; the DBG build of the check sets NETCSUM_TEST_DBG). */
#ifndef NET_CFG_MODULE_PRESENT
#define NET_CFG_MODULE_PRESENT
#include "lib_def.h"
#ifdef NETCSUM_TEST_DBG
#define NET_ERR_CFG_ARG_CHK_DBG_EN   DEF_ENABLED
#else
#define NET_ERR_CFG_ARG_CHK_DBG_EN   DEF_DISABLED
#endif
#ifdef NETCSUM_TEST_NO_EXT
#define NET_ERR_CFG_ARG_CHK_EXT_EN   DEF_DISABLED
#else
#define NET_ERR_CFG_ARG_CHK_EXT_EN   DEF_ENABLED   /* template default, Cfg/Template/net_cfg.h:178 */
#endif
#define NET_TCP_MODULE_EN                        /* net_cfg_net.h: TCP configured in */
#ifdef NETCSUM_TEST_OFFLOAD                      /* the burst adapters' build: every checksum offloaded */
#define NET_IPV4_CFG_CHK_SUM_OFFLOAD_RX_EN   DEF_ENABLED   /* Cfg/Template/net_cfg.h:669-682 */
#define NET_IPV4_CFG_CHK_SUM_OFFLOAD_TX_EN   DEF_ENABLED
#define NET_ICMP_CFG_CHK_SUM_OFFLOAD_RX_EN   DEF_ENABLED
#define NET_ICMP_CFG_CHK_SUM_OFFLOAD_TX_EN   DEF_ENABLED
#define NET_UDP_CFG_CHK_SUM_OFFLOAD_RX_EN    DEF_ENABLED
#define NET_UDP_CFG_CHK_SUM_OFFLOAD_TX_EN    DEF_ENABLED
#define NET_TCP_CFG_CHK_SUM_OFFLOAD_RX_EN    DEF_ENABLED
#define NET_TCP_CFG_CHK_SUM_OFFLOAD_TX_EN    DEF_ENABLED
#endif
#endif
