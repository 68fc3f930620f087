/* In-stack compile check: uC-CPU scalar types (see README.md). */
#ifndef CPU_CORE_MODULE_PRESENT
#define CPU_CORE_MODULE_PRESENT
#include <stdint.h>
#include "lib_def.h"
typedef uint8_t   CPU_INT08U;
typedef uint16_t  CPU_INT16U;
typedef uint32_t  CPU_INT32U;
typedef uint8_t   CPU_BOOLEAN;
typedef char      CPU_CHAR;
#endif
