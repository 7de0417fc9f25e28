// log.h — diagnostics (MV2AMD_DEBUG=1 enables debug lines; the reference's
// PRINT_DEBUG / MV2_DEBUG_* equivalent, channels/common/src/util/debug_utils.c)
#pragma once
#include <stdio.h>
#include <stdlib.h>

namespace mv2 {
int log_rank();
bool log_debug_on();
}  // namespace mv2

#define MV2_ERR(fmt, ...) fprintf(stderr, "[mv2amd rank %d] error: " fmt "\n", mv2::log_rank(), ##__VA_ARGS__)
#define MV2_FATAL(fmt, ...)                                                                            \
    do {                                                                                               \
        fprintf(stderr, "[mv2amd rank %d] fatal: " fmt "\n", mv2::log_rank(), ##__VA_ARGS__);        \
        fflush(stderr);                                                                                \
        abort();                                                                                       \
    } while (0)
#define MV2_DEBUG(fmt, ...)                                                                            \
    do {                                                                                               \
        if (mv2::log_debug_on()) fprintf(stderr, "[mv2amd rank %d] " fmt "\n", mv2::log_rank(), ##__VA_ARGS__); \
    } while (0)
