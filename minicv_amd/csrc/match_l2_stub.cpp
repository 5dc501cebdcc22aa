// Temporary until the MFMA L2 matcher lands.
#include "kernels.h"
#include "mcv_runtime.h"
namespace mcv {
int launch_match_l2(const float*, int, const float*, int, int, int*, float*, int*, float*, hipStream_t) {
    fail("cvMatchL2: MFMA L2 matcher not built yet");
}
}  // namespace mcv
