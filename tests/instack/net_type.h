/* In-stack compile check: Source/net_type.h:122,184-235 values (see README.md). */
#ifndef NET_TYPE_MODULE_PRESENT
#define NET_TYPE_MODULE_PRESENT
#include "cpu_core.h"
typedef CPU_INT16U NET_CHK_SUM;
typedef enum net_protocol_type {
    NET_PROTOCOL_TYPE_NONE           =  0,
    NET_PROTOCOL_TYPE_IP_V4          = 40,
    NET_PROTOCOL_TYPE_IP_V6_EXT_NONE = 48,
    NET_PROTOCOL_TYPE_ICMP_V4        = 60,
    NET_PROTOCOL_TYPE_ICMP_V6        = 61,
    NET_PROTOCOL_TYPE_IGMP           = 62,
    NET_PROTOCOL_TYPE_UDP_V4         = 70,
    NET_PROTOCOL_TYPE_TCP_V4         = 71,
    NET_PROTOCOL_TYPE_UDP_V6         = 72,
    NET_PROTOCOL_TYPE_TCP_V6         = 73
} NET_PROTOCOL_TYPE;
#endif
