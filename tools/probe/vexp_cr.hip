// vexp_cr.hip -- is the hardware v_exp_f32 (__builtin_amdgcn_exp2f) correctly rounded?
//
// Every negative float x with |x| <= 128 (bit patterns 0x80000000 .. 0xC3000000, 1.12e9 values)
// against the correctly rounded 2^x: exp2 in double rounded once to float. The double result is
// within 1 double ulp of 2^x, so the float rounding is correct unless 2^x lies within ~2^-29 float
// ulp of a rounding midpoint; those inputs are counted separately ("near-tie") and excluded.
// Output: mismatches per binade of x, the worst ulp distance, the first few examples, and the same
// for the blend's decision domain x in [-8, 0] (alpha = o 2^x >= 1/255 needs x >= -log2(255) > -8).
//   hipcc --offload-arch=gfx950 -O3 -o tools/probe/bin/vexp_cr tools/probe/vexp_cr.hip
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

struct Stats {
    unsigned long long mism_binade[256];
    unsigned long long near_tie;
    unsigned long long mism_decision;  // x in [-8, 0]
    unsigned long long checked;
    unsigned int max_ulp;
    unsigned int n_ex;
    uint32_t ex_x[64], ex_hw[64], ex_cr[64];
};

__global__ void probe(uint32_t lo, uint32_t n, Stats* s) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint32_t xb = lo + i;
    const float x = __uint_as_float(xb);
    const float hw = __builtin_amdgcn_exp2f(x);
    const double d = exp2((double)x);
    const float cr = (float)d;
    // distance of d from the float rounding midpoint, in units of the float ulp
    const double ulp = (double)(nextafterf(cr, INFINITY) - cr);
    const double frac = (d - (double)cr) / ulp;  // in (-0.5, 0.5]
    if (fabs(fabs(frac) - 0.5) < 1e-6) {
        atomicAdd(&s->near_tie, 1ull);
        return;
    }
    if (__float_as_uint(hw) != __float_as_uint(cr)) {
        const uint32_t e = (xb >> 23) & 0xff;
        atomicAdd(&s->mism_binade[e], 1ull);
        const int du = (int)__float_as_uint(hw) - (int)__float_as_uint(cr);
        atomicMax(&s->max_ulp, (unsigned)(du < 0 ? -du : du));
        if (x >= -8.0f) atomicAdd(&s->mism_decision, 1ull);
        const unsigned k = atomicAdd(&s->n_ex, 1u);
        if (k < 64) {
            s->ex_x[k] = xb;
            s->ex_hw[k] = __float_as_uint(hw);
            s->ex_cr[k] = __float_as_uint(cr);
        }
    }
}

static float as_f(uint32_t u) {
    float f;
    memcpy(&f, &u, 4);
    return f;
}

int main() {
    Stats* s;
    hipMalloc(&s, sizeof(Stats));
    hipMemset(s, 0, sizeof(Stats));
    const uint32_t lo = 0x80000000u, hi = 0xC3000000u;  // -0 .. -128
    const uint32_t chunk = 1u << 28;
    for (uint64_t b = lo; b <= hi; b += chunk) {
        const uint32_t n = (uint32_t)((hi + 1ull - b) < chunk ? (hi + 1ull - b) : chunk);
        hipLaunchKernelGGL(probe, dim3((n + 255) / 256), dim3(256), 0, 0, (uint32_t)b, n, s);
    }
    Stats h;
    hipMemcpy(&h, s, sizeof(Stats), hipMemcpyDeviceToHost);
    unsigned long long tot = 0;
    for (int e = 0; e < 256; ++e) tot += h.mism_binade[e];
    printf("{\"checked\": %llu, \"near_tie_excluded\": %llu, \"mismatches\": %llu, \"mismatches_x_ge_-8\": %llu, "
           "\"max_ulp\": %u,\n \"mismatch_by_binade\": {",
           (unsigned long long)(0xC3000000ull - 0x80000000ull + 1) - h.near_tie, h.near_tie, tot, h.mism_decision, h.max_ulp);
    bool first = true;
    for (int e = 0; e < 256; ++e)
        if (h.mism_binade[e]) {
            printf("%s\"2^%d\": %llu", first ? "" : ", ", e - 127, h.mism_binade[e]);
            first = false;
        }
    printf("},\n \"examples\": [");
    const unsigned ne = h.n_ex < 64 ? h.n_ex : 64;
    for (unsigned k = 0; k < ne; ++k)
        printf("%s[\"%a\", \"%a\", \"%a\"]", k ? ", " : "", as_f(h.ex_x[k]), as_f(h.ex_hw[k]), as_f(h.ex_cr[k]));
    printf("]}\n");
    return 0;
}
