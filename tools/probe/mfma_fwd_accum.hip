// Probe for the forward blend's MFMA accumulation (render_fwd.hip):
//  1. v_permlane32_swap + v_permlane16_swap as a 4x4 transpose of (register, 16-lane row): after
//     the swaps register m, row g must hold the original register g, row m;
//  2. v_mfma_f32_16x16x4f32 against a sequential fmaf chain over k = 0..3 (acc = fmaf(a_k, b_k,
//     acc) in k order): bitwise equal on inputs with heavy cancellation and mixed magnitudes?
//     Also the same with a zero A column (non-contributing pixel) and denormal products.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <cmath>
typedef float floatx4 __attribute__((ext_vector_type(4)));

__global__ void transpose_k(unsigned* out) {
    const int l = threadIdx.x;
    unsigned r[4];
    for (int k = 0; k < 4; ++k) r[k] = (unsigned)(k * 1000 + l);  // register k, lane l
    auto s02 = __builtin_amdgcn_permlane32_swap(r[0], r[2], false, false);
    r[0] = s02[0]; r[2] = s02[1];
    auto s13 = __builtin_amdgcn_permlane32_swap(r[1], r[3], false, false);
    r[1] = s13[0]; r[3] = s13[1];
    auto s01 = __builtin_amdgcn_permlane16_swap(r[0], r[1], false, false);
    r[0] = s01[0]; r[1] = s01[1];
    auto s23 = __builtin_amdgcn_permlane16_swap(r[2], r[3], false, false);
    r[2] = s23[0]; r[3] = s23[1];
    for (int k = 0; k < 4; ++k) out[k * 64 + l] = r[k];
}

// A: [16 m][4 k] per lane l = (m = l & 15, k = l >> 4); B: lane l = (k = l >> 4, n = l & 15);
// D: lane l holds rows 4 (l >> 4) + i, column l & 15. Chains of NCH MFMAs on one accumulator.
constexpr int NCH = 64;
__global__ void mfma_k(const float* A, const float* B, const float* C0, float* D) {
    const int l = threadIdx.x;
    floatx4 acc;
    for (int i = 0; i < 4; ++i) acc[i] = C0[(4 * (l >> 4) + i) * 16 + (l & 15)];
    for (int c = 0; c < NCH; ++c)
        acc = __builtin_amdgcn_mfma_f32_16x16x4f32(A[c * 64 + l], B[c * 64 + l], acc, 0, 0, 0);
    for (int i = 0; i < 4; ++i) D[(4 * (l >> 4) + i) * 16 + (l & 15)] = acc[i];
}

static float frand(unsigned& s) {
    s = s * 1664525u + 1013904223u;
    return ((s >> 8) * (1.0f / 16777216.0f)) * 2.f - 1.f;
}

int main() {
    unsigned *dt, ht[256];
    hipMalloc(&dt, sizeof(ht));
    hipLaunchKernelGGL(transpose_k, dim3(1), dim3(64), 0, 0, dt);
    hipMemcpy(ht, dt, sizeof(ht), hipMemcpyDeviceToHost);
    int ok = 1;
    for (int m = 0; m < 4; ++m)
        for (int l = 0; l < 64; ++l) {
            const int g = l >> 4, r = l & 15;
            if (ht[m * 64 + l] != (unsigned)(g * 1000 + (m * 16 + r))) ok = 0;
        }
    printf("permlane 4x4 transpose: %s (reg0 lanes 0,16,32,48: %u %u %u %u)\n", ok ? "CONFIRMED" : "REJECTED",
           ht[0], ht[16], ht[32], ht[48]);

    for (int trial = 0; trial < 3; ++trial) {
        unsigned s = 12345u + 777u * trial;
        float *hA = new float[NCH * 64], *hB = new float[NCH * 64], hC[256], hD[256], ref[256];
        for (int i = 0; i < NCH * 64; ++i) {
            float a = frand(s), b = frand(s);
            if (trial == 1) { a = ldexpf(a, (int)(frand(s) * 20)); b = ldexpf(b, (int)(frand(s) * 20)); }
            if (trial == 2) { if ((i % 7) == 0) a = 0.f; b = ldexpf(b, -120); }  // zero w, tiny products
            hA[i] = a; hB[i] = b;
        }
        for (int i = 0; i < 256; ++i) hC[i] = trial == 2 ? ldexpf(frand(s), -125) : frand(s) * 100.f;
        float *dA, *dB, *dC, *dD;
        hipMalloc(&dA, NCH * 64 * 4); hipMalloc(&dB, NCH * 64 * 4); hipMalloc(&dC, 1024); hipMalloc(&dD, 1024);
        hipMemcpy(dA, hA, NCH * 64 * 4, hipMemcpyHostToDevice);
        hipMemcpy(dB, hB, NCH * 64 * 4, hipMemcpyHostToDevice);
        hipMemcpy(dC, hC, 1024, hipMemcpyHostToDevice);
        hipLaunchKernelGGL(mfma_k, dim3(1), dim3(64), 0, 0, dA, dB, dC, dD);
        hipMemcpy(hD, dD, 1024, hipMemcpyDeviceToHost);
        int same = 0, same_rev = 0;
        for (int m = 0; m < 16; ++m)
            for (int n = 0; n < 16; ++n) {
                float acc = hC[m * 16 + n], accr = acc;
                for (int c = 0; c < NCH; ++c) {
                    for (int k = 0; k < 4; ++k) {
                        const float a = hA[c * 64 + k * 16 + m], b = hB[c * 64 + k * 16 + n];
                        acc = fmaf(a, b, acc);
                    }
                    for (int k = 3; k >= 0; --k) {
                        const float a = hA[c * 64 + k * 16 + m], b = hB[c * 64 + k * 16 + n];
                        accr = fmaf(a, b, accr);
                    }
                }
                ref[m * 16 + n] = acc;
                same += memcmp(&acc, &hD[m * 16 + n], 4) == 0;
                same_rev += memcmp(&accr, &hD[m * 16 + n], 4) == 0;
            }
        printf("trial %d: MFMA == fmaf chain k ascending: %d/256, k descending: %d/256 (D[0] %a ref %a)\n", trial,
               same, same_rev, hD[0], ref[0]);
    }
    return 0;
}
