/*
 * netcsum_types.h — the µC/TCP-IP scalar types and error codes the checksum ABI uses.
 *
 * When this header is compiled INSIDE a µC/TCP-IP build, the stack's own headers already define
 * these (define NETCSUM_HAVE_MICRIUM_TYPES before including netcsum_mi355x.h, or include
 * <net_util.h> first — it defines NET_UTIL_MODULE_PRESENT via net_util.h's include guard).
 * Standalone builds (this repo's tests, bench, Python bindings) get plain <stdint.h> mirrors.
 *
 * Values mirror the reference exactly:
 *   NET_CHK_SUM = CPU_INT16U                      Source/net_type.h:122
 *   NET_PROTOCOL_TYPE enum                        Source/net_type.h:184-235
 *   NET_ERR enum values used by the path          Source/net_err.h:73,122-126,193
 *   DEF_OK = 1, DEF_FAIL = 0 (uC-LIB lib_def.h, not vendored — values used throughout the
 *   reference, e.g. Source/net_util.c:276)
 *   NET_BUF_IX_NONE = DEF_INT_16U_MAX_VAL         Source/net_buf.h:274
 */
#ifndef NETCSUM_TYPES_H
#define NETCSUM_TYPES_H

#include <stdint.h>

#if !defined(NETCSUM_HAVE_MICRIUM_TYPES) && !defined(NET_UTIL_MODULE_PRESENT)

typedef uint8_t  CPU_INT08U;
typedef uint16_t CPU_INT16U;
typedef uint32_t CPU_INT32U;
typedef uint8_t  CPU_BOOLEAN;
typedef CPU_INT16U NET_CHK_SUM;

#ifndef DEF_OK
#define DEF_FAIL 0u
#define DEF_OK   1u
#endif

typedef enum net_protocol_type {
    NET_PROTOCOL_TYPE_NONE             = 0,
    NET_PROTOCOL_TYPE_IP_V4            = 40,
    NET_PROTOCOL_TYPE_IP_V6_EXT_NONE   = 48,
    NET_PROTOCOL_TYPE_ICMP_V4          = 60,
    NET_PROTOCOL_TYPE_ICMP_V6          = 61,
    NET_PROTOCOL_TYPE_IGMP             = 62,
    NET_PROTOCOL_TYPE_UDP_V4           = 70,
    NET_PROTOCOL_TYPE_TCP_V4           = 71,
    NET_PROTOCOL_TYPE_UDP_V6           = 72,
    NET_PROTOCOL_TYPE_TCP_V6           = 73
} NET_PROTOCOL_TYPE;

typedef enum net_err {
    NET_ERR_NONE                  =   1u,
    NET_ERR_FAULT_NULL_PTR        =  23u,
    NET_UTIL_ERR_NONE             = 200u,
    NET_UTIL_ERR_NULL_SIZE        = 210u,
    NET_UTIL_ERR_INVALID_PROTOCOL = 211u,
    NET_UTIL_ERR_BUF_TOO_SMALL    = 212u,
    NET_BUF_ERR_INVALID_IX        = 622u
} NET_ERR;

#define NET_BUF_IX_NONE 0xFFFFu

#endif /* !NETCSUM_HAVE_MICRIUM_TYPES */

/*
 * Error codes ADDED by the MI355X build (unused in the reference's NET_UTIL range 200-219,
 * Source/net_err.h:122-126). A device failure is reported, never papered over by a CPU path.
 */
#define NET_UTIL_ERR_MI355X_DEV        218u   /* HIP runtime / device failure (no GPU, launch error) */
#define NET_UTIL_ERR_MI355X_INVALID_ARG 219u  /* batch ABI argument out of the supported range      */

#endif /* NETCSUM_TYPES_H */
