/* In-stack compile check: uC-LIB lib_def.h values the drop-in uses (see README.md). */
#ifndef LIB_DEF_MODULE_PRESENT
#define LIB_DEF_MODULE_PRESENT
#define DEF_DISABLED            0u
#define DEF_ENABLED             1u
#define DEF_NO                  0u
#define DEF_YES                 1u
#define DEF_FAIL                0u
#define DEF_OK                  1u
#define DEF_INT_16U_MAX_VAL     65535u
#endif
