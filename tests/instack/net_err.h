/* In-stack compile check: the NET_ERR enum (Source/net_err.h:73,122-126,193, closed at :1127). The
 * real enum has ~400 members; this subset keeps their values. */
#ifndef NET_ERR_MODULE_PRESENT
#define NET_ERR_MODULE_PRESENT
typedef enum net_err {
    NET_ERR_NONE                  =   1u,
    NET_ERR_FAULT_NULL_PTR        =  23u,
    NET_UTIL_ERR_NONE             = 200u,
    NET_UTIL_ERR_NULL_PTR         = 201u,
    NET_UTIL_ERR_NULL_SIZE        = 210u,
    NET_UTIL_ERR_INVALID_PROTOCOL = 211u,
    NET_UTIL_ERR_BUF_TOO_SMALL    = 212u,
    NET_BUF_ERR_INVALID_IX        = 622u
} NET_ERR;
#endif
