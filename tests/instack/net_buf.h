/* In-stack compile check: a NET_BUF with the reference's field NAMES and types (net_buf.h:394-598)
 * but a layout that differs from the template mirror include/netcsum_netbuf.h — as a configuration
 * with IPv6 / extra fields would — so the check shows the drop-in binds by name, not by offset. */
#ifndef NET_BUF_MODULE_PRESENT
#define NET_BUF_MODULE_PRESENT
#include "cpu_core.h"
#include "net_type.h"
#define NET_BUF_IX_NONE  DEF_INT_16U_MAX_VAL                        /* net_buf.h:274 */
typedef CPU_INT16U NET_BUF_SIZE;                                     /* net_buf.h:272 */
typedef struct net_buf NET_BUF;
typedef struct net_buf_hdr {
    CPU_INT32U         Type;
    CPU_INT16U         Flags;
    CPU_INT08U         IPv6_AddrsSrc[16];      /* extra: not in the template layout */
    NET_BUF           *PrevBufPtr;
    NET_BUF           *NextBufPtr;
    NET_PROTOCOL_TYPE  ProtocolHdrType;
    NET_PROTOCOL_TYPE  ProtocolHdrTypeIF;
    CPU_INT16U         IP_HdrIx;
    CPU_INT16U         ICMP_MsgIx;
    CPU_INT16U         ICMP_MsgLen;
    CPU_INT16U         ICMP_HdrLen;
    CPU_INT08U         IPv6_ExtHdrs[40];       /* extra */
    CPU_INT16U         TransportHdrIx;
    CPU_INT16U         TransportHdrLen;
    CPU_INT16U         TransportTotLen;
    CPU_INT16U         TransportDataLen;
    CPU_INT16U         DataIx;
    NET_BUF_SIZE       DataLen;
    NET_BUF_SIZE       TotLen;
    void              *TmrPtr;
} NET_BUF_HDR;
struct net_buf {
    NET_BUF_HDR  Hdr;
    CPU_INT08U  *DataPtr;
};
#endif
