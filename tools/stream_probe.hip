// Streaming ceiling for the preprocess's traffic (measurement aid, round 6):
//   hipcc --offload-arch=gfx950 -O3 -o build/stream_probe tools/stream_probe.hip && build/stream_probe [P]
// k_pattern reads every Gaussian's inputs the way k_preprocess<kShDirect> does (per lane: 12-B means,
// 16-B rotation, 12-B scales, 4-B opacity, 12-B dc, the 180-B _features_rest row as 11 dwordx4 + 1
// dword) and writes its outputs (48-B record, depth, radius, tiles, 8-B rectangle, clamp bits) with
// one add per value in place of the arithmetic; k_coalesced moves the same bytes with consecutive
// lanes on consecutive 16-B words.  Prints the average time and GB/s of each over 50 launches.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CHECK(x)                                                                   \
    do {                                                                           \
        hipError_t e_ = (x);                                                       \
        if (e_ != hipSuccess) {                                                    \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                \
            exit(1);                                                               \
        }                                                                          \
    } while (0)

struct In {
    const float *means, *rots, *scales, *opac, *dc, *rest;
};
struct Out {
    float4* rec;
    uint32_t *depth, *radii, *tiles, *clamped;
    uint2* rect;
};

__global__ __launch_bounds__(128) void k_pattern(int P, In in, Out out)
{
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= P) return;
    const float* m = in.means + 3 * (size_t)i;
    const float4 q = *reinterpret_cast<const float4*>(in.rots + 4 * (size_t)i);
    const float* s = in.scales + 3 * (size_t)i;
    const float* d = in.dc + 3 * (size_t)i;
    const char* row = reinterpret_cast<const char*>(in.rest) + 180 * (size_t)i;
    float acc = m[0] + m[1] + m[2] + q.x + q.y + q.z + q.w + s[0] + s[1] + s[2] + in.opac[i] + d[0] + d[1] + d[2];
#pragma unroll
    for (int k = 0; k < 11; k++) {
        float4 v;
        __builtin_memcpy(&v, row + 16 * k, 16);
        acc += v.x + v.y + v.z + v.w;
    }
    acc += *reinterpret_cast<const float*>(row + 176);
    float4* r = out.rec + 3 * (size_t)i;
    r[0] = make_float4(acc, acc + 1.f, acc + 2.f, acc + 3.f);
    r[1] = make_float4(acc + 4.f, acc + 5.f, acc + 6.f, acc + 7.f);
    r[2] = make_float4(acc + 8.f, acc + 9.f, acc + 10.f, acc + 11.f);
    const uint32_t u = __float_as_uint(acc);
    out.depth[i] = u;
    out.radii[i] = u + 1u;
    out.tiles[i] = u + 2u;
    out.clamped[i] = u + 3u;
    out.rect[i] = make_uint2(u + 4u, u + 5u);
}

__global__ __launch_bounds__(256) void k_coalesced(int64_t n_in16, const float4* in, int64_t n_out16, float4* out)
{
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    float acc = 0.f;
    for (int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; k < n_in16; k += stride) {
        const float4 v = in[k];
        acc += v.x + v.y + v.z + v.w;
    }
    for (int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; k < n_out16; k += stride)
        out[k] = make_float4(acc, acc, acc, acc);
}

int main(int argc, char** argv)
{
    const int P = argc > 1 ? atoi(argv[1]) : 1000000;
    const size_t in_floats = (size_t)P * (3 + 4 + 3 + 1 + 3 + 45);
    const size_t out_bytes = (size_t)P * (48 + 4 * 4 + 8);
    float* inbuf;
    char* outbuf;
    CHECK(hipMalloc(&inbuf, in_floats * 4 + 256));
    CHECK(hipMalloc(&outbuf, out_bytes + 256));
    CHECK(hipMemset(inbuf, 0, in_floats * 4));
    In in;
    float* p = inbuf;
    in.means = p;
    p += 3 * (size_t)P;
    in.rots = p;
    p += 4 * (size_t)P;
    in.scales = p;
    p += 3 * (size_t)P;
    in.opac = p;
    p += (size_t)P;
    in.dc = p;
    p += 3 * (size_t)P;
    in.rest = p;
    Out out;
    char* o = outbuf;
    out.rec = reinterpret_cast<float4*>(o);
    o += 48 * (size_t)P;
    out.depth = reinterpret_cast<uint32_t*>(o);
    o += 4 * (size_t)P;
    out.radii = reinterpret_cast<uint32_t*>(o);
    o += 4 * (size_t)P;
    out.tiles = reinterpret_cast<uint32_t*>(o);
    o += 4 * (size_t)P;
    out.clamped = reinterpret_cast<uint32_t*>(o);
    o += 4 * (size_t)P;
    out.rect = reinterpret_cast<uint2*>(o);
    const double bytes = (double)in_floats * 4 + (double)out_bytes;
    hipEvent_t a, b;
    CHECK(hipEventCreate(&a));
    CHECK(hipEventCreate(&b));
    for (int variant = 0; variant < 2; variant++) {
        for (int rep = 0; rep < 3; rep++) {
            const int iters = 50;
            for (int w = 0; w < 5; w++) {
                if (variant == 0) hipLaunchKernelGGL(k_pattern, dim3((P + 127) / 128), dim3(128), 0, 0, P, in, out);
                else hipLaunchKernelGGL(k_coalesced, dim3(2048), dim3(256), 0, 0, (int64_t)(in_floats / 4),
                                        reinterpret_cast<const float4*>(inbuf), (int64_t)(out_bytes / 16),
                                        reinterpret_cast<float4*>(outbuf));
            }
            CHECK(hipEventRecord(a, 0));
            for (int it = 0; it < iters; it++) {
                if (variant == 0) hipLaunchKernelGGL(k_pattern, dim3((P + 127) / 128), dim3(128), 0, 0, P, in, out);
                else hipLaunchKernelGGL(k_coalesced, dim3(2048), dim3(256), 0, 0, (int64_t)(in_floats / 4),
                                        reinterpret_cast<const float4*>(inbuf), (int64_t)(out_bytes / 16),
                                        reinterpret_cast<float4*>(outbuf));
            }
            CHECK(hipEventRecord(b, 0));
            CHECK(hipEventSynchronize(b));
            float ms = 0.f;
            CHECK(hipEventElapsedTime(&ms, a, b));
            const double us = 1000.0 * ms / iters;
            printf("stream_probe P=%d %s: %.1f us per launch, %.0f MB, %.2f TB/s\n", P,
                   variant == 0 ? "preprocess pattern" : "coalesced        ", us, bytes / 1e6, bytes / us / 1e6);
        }
    }
    CHECK(hipFree(inbuf));
    CHECK(hipFree(outbuf));
    return 0;
}
