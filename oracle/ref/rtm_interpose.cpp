// rtm_interpose.cpp — TEST INFRASTRUCTURE ONLY. Linked into oracle/_ref/libref_rtm.so (with
// -fno-builtin -Wl,-Bsymbolic) so the reference's calls to acosf/sinf/cosf/atan2f resolve to the
// shared bit-reproducible functions the GPU build uses (SURVEY.md §8c "interposition"). The
// reference code itself is untouched; only the C library it links against changes.
#include "../../include/rtg_math.h"

extern "C" {
float acosf(float x) { return rtm_acosf(x); }
float sinf(float x) { return rtm_sinf(x); }
float cosf(float x) { return rtm_cosf(x); }
float atan2f(float y, float x) { return rtm_atan2f(y, x); }
}
