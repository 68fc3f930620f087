/* In-stack compile check: the declarations of Source/net_util.h the drop-in implements. The
 * prototypes are the reference's (net_util.h:422-450; tests/test_boundary_cpu.py compares them token
 * for token with the reference header when /root/reference is present). */
#ifndef NET_UTIL_MODULE_PRESENT
#define NET_UTIL_MODULE_PRESENT
#include "cpu_core.h"
#include "net_cfg.h"
#include "net_type.h"
#include "net_err.h"

#define  NET_UTIL_NET_TO_HOST_16(val)   ((CPU_INT16U)__builtin_bswap16((CPU_INT16U)(val)))   /* LE host */

NET_CHK_SUM  NetUtil_16BitOnesCplChkSumHdrCalc   (void        *phdr,
                                                  CPU_INT16U   hdr_size,
                                                  NET_ERR     *p_err);

CPU_BOOLEAN  NetUtil_16BitOnesCplChkSumHdrVerify (void        *phdr,
                                                  CPU_INT16U   hdr_size,
                                                  NET_ERR     *p_err);

NET_CHK_SUM  NetUtil_16BitOnesCplChkSumDataCalc  (void        *pdata_buf,
                                                  void        *ppseudo_hdr,
                                                  CPU_INT16U   pseudo_hdr_size,
                                                  NET_ERR     *p_err);

CPU_BOOLEAN  NetUtil_16BitOnesCplChkSumDataVerify(void        *pdata_buf,
                                                  void        *ppseudo_hdr,
                                                  CPU_INT16U   pseudo_hdr_size,
                                                  NET_ERR     *p_err);

CPU_INT32U  NetUtil_16BitSumDataCalcAlign_32(void        *pdata_32,
                                             CPU_INT32U   size);

CPU_INT32U   NetUtil_32BitCRC_Calc               (CPU_INT08U  *p_data,
                                                  CPU_INT32U   data_len,
                                                  NET_ERR     *p_err);

CPU_INT32U   NetUtil_32BitCRC_CalcCpl            (CPU_INT08U  *p_data,
                                                  CPU_INT32U   data_len,
                                                  NET_ERR     *p_err);

CPU_INT32U   NetUtil_32BitReflect                (CPU_INT32U   val);
#endif
