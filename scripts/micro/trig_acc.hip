// Accuracy of gfx950's hardware v_sin_f32 / v_cos_f32 (argument in revolutions, scaled by
// 1/(2 pi) in f32) against f64 libm, for the joint angle range of the RK4 stages (|q1| <= 3.2
// rad: the joint-1 limit is +-3) and wider ranges; and of rd_physics.h's sincos_acc for
// comparison.  Prints the max absolute error per range.  hipcc --offload-arch=gfx950 -O3.
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdio.h>
#include <stdlib.h>

#include "../../reacherdistilation_amd/csrc/rd_physics.h"

__global__ void trig(const float* x, float* s_hw, float* c_hw, float* s_sw, float* c_sw, float* s_q0, float* c_q0, int n) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    const float r = x[i] * 0.15915494309189535f;   // 1 / (2 pi)
    s_hw[i] = __builtin_amdgcn_sinf(r);
    c_hw[i] = __builtin_amdgcn_cosf(r);
    float s, c;
    rd::sincos_acc<false>(x[i], &s, &c);
    s_sw[i] = s;
    c_sw[i] = c;
    rd::sincos_q0<false>(x[i], &s, &c);   // 2 pi Cody-Waite + the hardware
    s_q0[i] = s;
    c_q0[i] = c;
}

int main() {
    const int n = 1 << 22;
    const float ranges[] = {0.5f, 3.2f, 10.0f, 50.0f, 200.0f, 2000.0f};
    float *x, *o[6];
    (void)hipMallocManaged(&x, n * 4);
    for (int k = 0; k < 6; ++k) (void)hipMallocManaged(&o[k], n * 4);
    for (float R : ranges) {
        srand(1);
        for (int i = 0; i < n; ++i) x[i] = (float)((2.0 * rand() / RAND_MAX - 1.0) * R);
        hipLaunchKernelGGL(trig, dim3((n + 255) / 256), dim3(256), 0, 0, x, o[0], o[1], o[2], o[3], o[4], o[5], n);
        (void)hipDeviceSynchronize();
        double e[6] = {0, 0, 0, 0, 0, 0};
        for (int i = 0; i < n; ++i) {
            const double s = sin((double)x[i]), c = cos((double)x[i]);
            e[0] = fmax(e[0], fabs(o[0][i] - s)); e[1] = fmax(e[1], fabs(o[1][i] - c));
            e[2] = fmax(e[2], fabs(o[2][i] - s)); e[3] = fmax(e[3], fabs(o[3][i] - c));
            e[4] = fmax(e[4], fabs(o[4][i] - s)); e[5] = fmax(e[5], fabs(o[5][i] - c));
        }
        printf("{\"range_rad\": %g, \"hw_sin\": %.3e, \"hw_cos\": %.3e, \"sincos_acc_sin\": %.3e, \"sincos_acc_cos\": %.3e, \"sincos_q0_sin\": %.3e, \"sincos_q0_cos\": %.3e}\n",
               R, e[0], e[1], e[2], e[3], e[4], e[5]);
    }
    return 0;
}
