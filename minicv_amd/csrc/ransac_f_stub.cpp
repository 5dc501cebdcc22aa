// Temporary: fundamental-matrix family not built yet.
#include "plan.h"
namespace mcv {
void f_evaluate_chunk(Plan&, const float*, int, const RansacConfig&, int64_t, int, int*, hipStream_t) {
    fail("fundamental-matrix RANSAC not implemented yet");
}
int f_finalize(Plan&, const float*, int, const RansacConfig&, int64_t, double*, uint8_t*, hipStream_t) {
    fail("fundamental-matrix RANSAC not implemented yet");
}
int f_fit_all(Plan&, const float*, int, hipStream_t, double*) {
    fail("fundamental-matrix fit not implemented yet");
}
int f_host_hypothesis(const float*, int, uint64_t, int64_t, double*, float*, int*) {
    fail("fundamental-matrix RANSAC not implemented yet");
}
}  // namespace mcv
