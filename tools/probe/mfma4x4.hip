// Probe of the v_mfma_f32_4x4x1f32 (16-block) operand layout: A = lane id, B = 1000 * lane id.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef float floatx4 __attribute__((ext_vector_type(4)));
__global__ void k(float* out) {
    const int l = threadIdx.x;
    floatx4 c = {0.f, 0.f, 0.f, 0.f};
    floatx4 d = __builtin_amdgcn_mfma_f32_4x4x1f32((float)(l + 1), (float)(1000 * (l + 1)), c, 0, 0, 0);
    for (int r = 0; r < 4; ++r) out[l * 4 + r] = d[r];
}
int main() {
    float* d;
    hipMalloc(&d, 256 * sizeof(float));
    hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d);
    float h[256];
    hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
    int ok = 1;
    for (int l = 0; l < 64; ++l)
        for (int r = 0; r < 4; ++r) {
            // expected: block b = l/4, row r, col l%4: A from lane 4b + r, B from lane 4b + l%4
            const int b = l / 4;
            const float e = (float)(4 * b + r + 1) * 1000.f * (float)(4 * b + (l % 4) + 1);
            if (h[l * 4 + r] != e) ok = 0;
        }
    printf("lane0: %g %g %g %g  lane5: %g %g %g %g\n", h[0], h[1], h[2], h[3], h[20], h[21], h[22], h[23]);
    printf("layout hypothesis %s\n", ok ? "CONFIRMED" : "REJECTED");
    return 0;
}
