// Microbenchmark: cycles per serial step of the 64-row insertion chain x_i = (m_i + x_{i-1} k_i) + d_i
// (fill_coop.hip insertion_chain, G = 64).  A: DPP wave_shr:1 hand-off (current); B: operands moved to
// SGPRs with v_readlane, every lane runs the chain on uniform operands, lane q keeps step q's value.
#include <hip/hip_runtime.h>
#include <cstdio>

template <int CTRL, int ROWMASK, bool BOUND>
__device__ __forceinline__ double dpp_d(double old, double x)
{
    const int xl = __double2loint(x), xh = __double2hiint(x);
    const int ol = __double2loint(old), oh = __double2hiint(old);
    const int rl = __builtin_amdgcn_update_dpp(ol, xl, CTRL, ROWMASK, 0xF, BOUND);
    const int rh = __builtin_amdgcn_update_dpp(oh, xh, CTRL, ROWMASK, 0xF, BOUND);
    return __hiloint2double(rh, rl);
}

__device__ __forceinline__ double rl(double v, int q)
{
    const int lo = __builtin_amdgcn_readlane(__double2loint(v), q);
    const int hi = __builtin_amdgcn_readlane(__double2hiint(v), q);
    return __hiloint2double(hi, lo);
}

__global__ void __launch_bounds__(64) kA(const double* in, double* out, long long* cyc, int chunks)
{
    const int lane = threadIdx.x;
    double m = in[lane], k = in[64 + lane], d = in[128 + lane];
    double carry = 1.0, acc = 0.0;
    const long long c0 = clock64();
    for (int c = 0; c < chunks; ++c) {
        double x = 0.0, up = carry;
#pragma unroll
        for (int q = 0; q < 64; ++q) {
            up = dpp_d<0x138, 0xF, false>(up, x);
            x = (m + up * k) + d;
        }
        carry = __shfl(x, 63);
        acc += x;
        m = m * 0.5 + 1e-3;
    }
    const long long c1 = clock64();
    out[lane] = acc;
    if (lane == 0) cyc[blockIdx.x] = c1 - c0;
}

__global__ void __launch_bounds__(64) kB(const double* in, double* out, long long* cyc, int chunks)
{
    const int lane = threadIdx.x;
    double m = in[lane], k = in[64 + lane], d = in[128 + lane];
    double carry = 1.0, acc = 0.0;
    const long long c0 = clock64();
    for (int c = 0; c < chunks; ++c) {
        double x = carry, mine = 0.0;
#pragma unroll
        for (int q = 0; q < 64; ++q) {
            const double mq = rl(m, q), kq = rl(k, q), dq = rl(d, q);
            x = (mq + x * kq) + dq;
            mine = lane == q ? x : mine;
        }
        carry = x;
        acc += mine;
        m = m * 0.5 + 1e-3;
    }
    const long long c1 = clock64();
    out[lane] = acc;
    if (lane == 0) cyc[blockIdx.x] = c1 - c0;
}

int main()
{
    double h[192];
    for (int i = 0; i < 192; ++i) h[i] = 0.001 * (i % 64) + (i >= 64 && i < 128 ? 0.01 : 0.1);
    double *din, *dout;
    long long* dc;
    hipMalloc(&din, sizeof(h));
    hipMalloc(&dout, 64 * 8 * 2);
    hipMalloc(&dc, 8 * 1024 * sizeof(long long));
    hipMemcpy(din, h, sizeof(h), hipMemcpyHostToDevice);
    const int chunks = 2000;
    for (int blocks : {1, 256, 1024, 2048}) {
        long long cyc[2048];
        double oa[64], ob[64];
        hipLaunchKernelGGL(kA, dim3(blocks), dim3(64), 0, 0, din, dout, dc, chunks);
        hipMemcpy(cyc, dc, blocks * sizeof(long long), hipMemcpyDeviceToHost);
        hipMemcpy(oa, dout, sizeof(oa), hipMemcpyDeviceToHost);
        long long a = 0;
        for (int b = 0; b < blocks; ++b) a += cyc[b];
        hipLaunchKernelGGL(kB, dim3(blocks), dim3(64), 0, 0, din, dout, dc, chunks);
        hipMemcpy(cyc, dc, blocks * sizeof(long long), hipMemcpyDeviceToHost);
        hipMemcpy(ob, dout, sizeof(ob), hipMemcpyDeviceToHost);
        long long b2 = 0;
        for (int b = 0; b < blocks; ++b) b2 += cyc[b];
        int same = 1;
        for (int i = 0; i < 64; ++i) same &= (oa[i] == ob[i]);
        printf("blocks %5d: A dpp %.1f cyc/step   B readlane %.1f cyc/step   bit-identical %d\n", blocks,
               (double)a / blocks / (chunks * 64.0), (double)b2 / blocks / (chunks * 64.0), same);
    }
    return 0;
}
