// Microbenchmark: cycles per band row of the in-column insertion chain x_i = (m_i + x_{i-1} k_i) + d_i
// (fill_coop.hip / coop_chain.hpp).  Every variant computes the same rows in the reference's operation order,
// so their outputs are compared bit for bit against A.
//   A    one row per lane, DPP wave_shr:1 hand-off per row (the current 64-lane chain)
//   B    operands moved to SGPRs with v_readlane, every lane runs the chain on uniform operands
//   C<R> R consecutive rows per lane: R register steps, then one wave_shr:1 hand-off (64 R rows per chunk)
//   D    two chains per wave in 32-lane halves: wave_shr:1 plus a select that restores lane 32's own carry
//   E    four chains per wave in 16-lane DPP rows (row_shr:1, the 16-lane fill's chain), per row of one chain
//   L    no hand-off at all: one lane-local chain of 3 dependent FP64 operations per row (the floor)
// Output: cycles per row (s_memtime, shader clock) at 1, 256, 1024 and 2048 waves.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstring>

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

__device__ __forceinline__ double last_lane(double x) { return rl(x, 63); }

// row r of the chunk sequence: inputs for row (c * rows + r), rows of a chunk = `rows`
__device__ __forceinline__ void inputs(const double* in, int row, double& m, double& k, double& d)
{
    const int q = row & 63;
    m = in[q];
    k = in[64 + q];
    d = in[128 + q];
}

// A: the current chain.  Output: per chunk, every row's value written to out[chunk-local row]
__global__ void __launch_bounds__(64) kA(const double* in, double* out, long long* cyc, int chunks, int rowsOut)
{
    const int lane = threadIdx.x;
    double m, k, d;
    inputs(in, lane, m, k, d);
    double carry = 1.0, acc = 0.0;
    const long long c0 = clock64();
    for (int c = 0; c < chunks; ++c) {
        double x = 0.0, up = carry;
#pragma unroll
        for (int q = 0; q < 64; ++q) {
            up = dpp_d<0x138, 0xF, false>(up, x);
            x = (m + up * k) + d;
        }
        carry = last_lane(x);
        acc += x;
        m = m * 0.5 + 1e-3;
    }
    const long long c1 = clock64();
    if (blockIdx.x == 0) out[lane] = acc;
    if (lane == 0) cyc[blockIdx.x] = c1 - c0;
    (void)rowsOut;
}

__global__ void __launch_bounds__(64) kB(const double* in, double* out, long long* cyc, int chunks, int rowsOut)
{
    const int lane = threadIdx.x;
    double m, k, d;
    inputs(in, lane, m, k, d);
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
    if (blockIdx.x == 0) out[lane] = acc;
    if (lane == 0) cyc[blockIdx.x] = c1 - c0;
    (void)rowsOut;
}

// C<R>: lane l owns rows [l R, l R + R) of a 64 R-row chunk.  The inputs are laid out so that the row
// sequence equals A's: chunk-row s = l R + r takes A's lane (s & 63) inputs and A's chunk index (s >> 6) gets the
// same m update, so the value of every row is A's bit for bit.
template <int R>
__global__ void __launch_bounds__(64) kC(const double* in, double* out, long long* cyc, int chunks, int rowsOut)
{
    const int lane = threadIdx.x;
    double m[R], k[R], d[R];
#pragma unroll
    for (int r = 0; r < R; ++r) inputs(in, lane * R + r, m[r], k[r], d[r]);
    // the m update of A happens once per 64 rows: row s of A's chunk c has m0 * 0.5^c + ...; reproduce by
    // applying the update to the rows whose A-chunk advanced
    double carry = 1.0, acc = 0.0;
    const long long c0 = clock64();
    for (int c = 0; c < chunks; c += R) {
        double x[R];
#pragma unroll
        for (int r = 0; r < R; ++r) x[r] = 0.0;
        double up = carry;
#pragma unroll
        for (int p = 0; p < 64; ++p) {
            up = dpp_d<0x138, 0xF, false>(up, x[R - 1]);
            x[0] = (m[0] + up * k[0]) + d[0];
#pragma unroll
            for (int r = 1; r < R; ++r) x[r] = (m[r] + x[r - 1] * k[r]) + d[r];
        }
        carry = last_lane(x[R - 1]);
#pragma unroll
        for (int r = 0; r < R; ++r) acc += x[r];
#pragma unroll
        for (int r = 0; r < R; ++r) m[r] = m[r] * 0.5 + 1e-3;
    }
    const long long c1 = clock64();
    if (blockIdx.x == 0) out[lane] = acc;
    if (lane == 0) cyc[blockIdx.x] = c1 - c0;
    (void)rowsOut;
}

// D: two independent 32-row chains per wave (lanes 0-31, 32-63); wave_shr:1 then lane 32 takes its own carry
__global__ void __launch_bounds__(64) kD(const double* in, double* out, long long* cyc, int chunks, int rowsOut)
{
    const int lane = threadIdx.x;
    double m, k, d;
    inputs(in, lane, m, k, d);
    double carry = 1.0, acc = 0.0;
    const bool head = (lane & 31) == 0;
    const long long c0 = clock64();
    for (int c = 0; c < chunks; ++c) {
        double x = 0.0, up = carry;
#pragma unroll
        for (int q = 0; q < 32; ++q) {
            const double s = dpp_d<0x138, 0xF, false>(up, x);
            up = head ? carry : s;
            x = (m + up * k) + d;
        }
        carry = (lane < 32) ? rl(x, 31) : rl(x, 63);
        acc += x;
        m = m * 0.5 + 1e-3;
    }
    const long long c1 = clock64();
    if (blockIdx.x == 0) out[lane] = acc;
    if (lane == 0) cyc[blockIdx.x] = c1 - c0;
    (void)rowsOut;
}

// E: four 16-row chains per wave (row_shr:1 leaves each DPP row's lane 0 with `old`)
__global__ void __launch_bounds__(64) kE(const double* in, double* out, long long* cyc, int chunks, int rowsOut)
{
    const int lane = threadIdx.x;
    double m, k, d;
    inputs(in, lane, m, k, d);
    double carry = 1.0, acc = 0.0;
    const long long c0 = clock64();
    for (int c = 0; c < chunks; ++c) {
        double x = 0.0, up = carry;
#pragma unroll
        for (int q = 0; q < 16; ++q) {
            up = dpp_d<0x111, 0xF, false>(up, x);
            x = (m + up * k) + d;
        }
        const long long r = __builtin_amdgcn_update_dpp(0ll, __double_as_longlong(x), 0x15F, 0xF, 0xF, false);
        carry = __longlong_as_double(r);
        acc += x;
        m = m * 0.5 + 1e-3;
    }
    const long long c1 = clock64();
    if (blockIdx.x == 0) out[lane] = acc;
    if (lane == 0) cyc[blockIdx.x] = c1 - c0;
    (void)rowsOut;
}

// L: the floor -- one lane-local chain, 64 rows per chunk, no cross-lane traffic
__global__ void __launch_bounds__(64) kL(const double* in, double* out, long long* cyc, int chunks, int rowsOut)
{
    const int lane = threadIdx.x;
    double m[8], k[8], d[8];
#pragma unroll
    for (int r = 0; r < 8; ++r) inputs(in, lane + r, m[r], k[r], d[r]);
    double x = 1.0, acc = 0.0;
    const long long c0 = clock64();
    for (int c = 0; c < chunks; ++c) {
#pragma unroll
        for (int q = 0; q < 64; ++q) x = (m[q & 7] + x * k[q & 7]) + d[q & 7];
        acc += x;
        m[c & 7] = m[c & 7] * 0.5 + 1e-3;
    }
    const long long c1 = clock64();
    if (blockIdx.x == 0) out[lane] = acc;
    if (lane == 0) cyc[blockIdx.x] = c1 - c0;
    (void)rowsOut;
}

using Kern = void (*)(const double*, double*, long long*, int, int);

static double run(Kern k, int blocks, int chunks, const double* din, double* dout, long long* dc, double* host64,
                  double rowsPerChunkPerWave)
{
    static long long cyc[4096];
    hipLaunchKernelGGL(k, dim3(blocks), dim3(64), 0, 0, din, dout, dc, chunks, 0);
    hipDeviceSynchronize();
    hipLaunchKernelGGL(k, dim3(blocks), dim3(64), 0, 0, din, dout, dc, chunks, 0);
    hipMemcpy(cyc, dc, blocks * sizeof(long long), hipMemcpyDeviceToHost);
    if (host64) hipMemcpy(host64, dout, 64 * sizeof(double), hipMemcpyDeviceToHost);
    double a = 0;
    for (int b = 0; b < blocks; ++b) a += (double)cyc[b];
    return a / blocks / (chunks * rowsPerChunkPerWave);
}

int main()
{
    double h[192];
    for (int i = 0; i < 192; ++i) h[i] = 0.001 * (i % 64) + (i >= 64 && i < 128 ? 0.01 : 0.1);
    double *din, *dout;
    long long* dc;
    hipMalloc(&din, sizeof(h));
    hipMalloc(&dout, 64 * 8 * 2);
    hipMalloc(&dc, 8 * 4096 * sizeof(long long));
    hipMemcpy(din, h, sizeof(h), hipMemcpyHostToDevice);
    const int chunks = 2048;   // a multiple of every R
    std::printf("cycles per chain row (one chain's row); lower is better\n");
    std::printf("%-34s %8s %8s %8s %8s\n", "variant", "1 wave", "256", "1024", "2048");
    struct V {
        const char* name;
        Kern k;
        double rowsPerChunk;   // rows of ONE chain per chunk iteration
    } vs[] = {
        {"A  64 lanes, DPP per row", kA, 64},
        {"B  readlane operands", kB, 64},
        {"C2 2 rows/lane, DPP per 2 rows", kC<2>, 128.0 / 2},
        {"C4 4 rows/lane, DPP per 4 rows", kC<4>, 256.0 / 4},
        {"C8 8 rows/lane, DPP per 8 rows", kC<8>, 512.0 / 8},
        {"D  2 chains x 32 lanes", kD, 32},
        {"E  4 chains x 16 lanes (row_shr)", kE, 16},
        {"L  lane-local, no hand-off", kL, 64},
    };
    double ref[64];
    for (const V& v : vs) {
        double o[64];
        std::printf("%-34s", v.name);
        for (int blocks : {1, 256, 1024, 2048}) {
            // C<R> iterates chunks / R times, each 64 R rows: per chain row it is chunks * 64 rows in all
            const double c = run(v.k, blocks, chunks, din, dout, dc, o, v.rowsPerChunk);
            std::printf(" %8.1f", c);
        }
        if (v.k == kA) std::memcpy(ref, o, sizeof(ref));
        std::printf("\n");
    }
    // bit-identity of C<R> against A: same row sequence, same operation order
    {
        double o[64];
        int same = 1;
        (void)run(kC<1>, 1, chunks, din, dout, dc, o, 64);
        for (int i = 0; i < 64; ++i) same &= (o[i] == ref[i]);
        std::printf("C1 == A bit for bit: %d\n", same);
    }
    return 0;
}
