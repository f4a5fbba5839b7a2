/* CPU ORACLE -- test infrastructure, NOT product code.
 *
 * Plain-C restatement of the reference's mu-law companding + mid-rise quantizer
 * (the integer/index part of the hot path):
 *   ulaw     utils.py:33-36   y = sign(x) * log(255|x| + 1) / 5.5451774444795623
 *   midrise  utils.py:48-51   i = (long)(0.5*(y+1) * (q - 1e-6))   (trunc toward 0)
 *   iulaw    utils.py:39-42   x = sign(c) * (exp(|c| * LOG_MU1) - 1) / 255
 *   imidrise utils.py:54-55   c = k * 2 / q - 1
 * evaluated in the dtype of the input exactly as torch does it:  float32 inputs in
 * float32 arithmetic (python-float scalars rounded to float first), float64 in double.
 * Only tests/ may load this library (as the checker); pinned against the reference's
 * own outputs in tests/golden/ulaw.npz by tests/test_oracle_golden.py.
 */
#include <math.h>
#include <stdint.h>

#define LOG_MU1_D 5.5451774444795623
#define MU_D 255.0

static inline double sgn_d(double x) { return (x > 0) - (x < 0); }
static inline float sgn_f(float x) { return (float)((x > 0) - (x < 0)); }

int64_t oracle_uquantize_f64(double x, int q_levels) {
    double y = sgn_d(x) * log(MU_D * fabs(x) + 1.0) / LOG_MU1_D;
    y = 0.5 * (y + 1.0);
    y *= ((double)q_levels - 1e-6);
    return (int64_t)y;
}

int64_t oracle_uquantize_f32(float x, int q_levels) {
    const float mu = (float)MU_D, lm = (float)LOG_MU1_D;
    const float scale = (float)((double)q_levels - 1e-6);
    float y = sgn_f(x) * logf(mu * fabsf(x) + 1.0f) / lm;
    y = 0.5f * (y + 1.0f);
    y *= scale;
    return (int64_t)y;
}

float oracle_udequantize(int64_t k, int q_levels) {
    float c = (float)k * 2.0f / (float)q_levels - 1.0f;
    float x = expf(fabsf(c) * (float)LOG_MU1_D) - 1.0f;
    return sgn_f(c) * x / (float)MU_D;
}

void oracle_uquantize_f64_n(const double* x, int64_t* out, int64_t n, int q) {
    for (int64_t i = 0; i < n; ++i) out[i] = oracle_uquantize_f64(x[i], q);
}
void oracle_uquantize_f32_n(const float* x, int64_t* out, int64_t n, int q) {
    for (int64_t i = 0; i < n; ++i) out[i] = oracle_uquantize_f32(x[i], q);
}
void oracle_udequantize_n(const int64_t* k, float* out, int64_t n, int q) {
    for (int64_t i = 0; i < n; ++i) out[i] = oracle_udequantize(k[i], q);
}
