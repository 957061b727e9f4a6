// FETCH_SIZE / WRITE_SIZE calibration on known byte counts (measurement aid,
// not the product). MI355X_MICROARCH.md calibrates FETCH_SIZE only for 16 B/lane
// streaming reads (it reports half the bytes); the headline kernels gather
// 64-byte NodeRecs and 1-8 byte columns through the visit order and write
// 8-byte values. Each pattern below touches a known set of unique bytes once
// (every row exactly once, in the same 64-lane workgroup shape as k_base);
// run the binary under two rocprofv3 passes (--pmc FETCH_SIZE, --pmc
// WRITE_SIZE) and divide the counters by the printed unique bytes
// (tools/fetch_calib.py does both).
//
// usage: fetch_calib [rows]   (default 10000, the headline cluster; 1<<20 too)
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <numeric>
#include <random>
#include <vector>

#define CK(x)                                                                    \
    do {                                                                         \
        hipError_t e_ = (x);                                                     \
        if (e_ != hipSuccess) {                                                  \
            std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));         \
            std::exit(1);                                                        \
        }                                                                        \
    } while (0)

struct alignas(16) Rec64 { uint4 q[4]; };

// a value the compiler cannot prove unused: stored only when it matches a
// sentinel the data never holds
__device__ __forceinline__ void keep(uint32_t v, uint32_t* sink) {
    if (v == 0xDEADBEEFu) sink[0] = v;
}

// 16 B per lane, coalesced (the guide's calibrated case)
__global__ void __launch_bounds__(64) c_stream16(const uint4* src, uint32_t n16, uint32_t* sink) {
    const uint32_t stride = gridDim.x * 64;
    uint32_t acc = 0;
    for (uint32_t i = blockIdx.x * 64 + threadIdx.x; i < n16; i += stride) {
        const uint4 v = src[i];
        acc ^= v.x ^ v.y ^ v.z ^ v.w;
    }
    keep(acc, sink);
}

// 64-byte records read in row order, one lane per record (4 x 16 B per lane)
__global__ void __launch_bounds__(64) c_rows64(const Rec64* tab, uint32_t rows, uint32_t* sink) {
    const uint32_t stride = gridDim.x * 64;
    uint32_t acc = 0;
    for (uint32_t j = blockIdx.x * 64 + threadIdx.x; j < rows; j += stride) {
        const Rec64 r = tab[j];
        for (int k = 0; k < 4; k++) acc ^= r.q[k].x ^ r.q[k].w;
    }
    keep(acc, sink);
}

// 64-byte records gathered through a permutation (k_base's visit-order read);
// PAIR: two neighbouring lanes read the same record (k_base's base / base1)
template <bool PAIR>
__global__ void __launch_bounds__(64) c_gather64(const Rec64* tab, const uint32_t* perm, uint32_t rows,
                                                 uint32_t* sink) {
    const uint32_t total = PAIR ? 2 * rows : rows;
    const uint32_t stride = gridDim.x * 64;
    uint32_t acc = 0;
    for (uint32_t t = blockIdx.x * 64 + threadIdx.x; t < total; t += stride) {
        const uint32_t row = perm[PAIR ? t >> 1 : t];
        const Rec64 r = tab[row];
        for (int k = 0; k < 4; k++) acc ^= r.q[k].x ^ r.q[k].w;
    }
    keep(acc, sink);
}

// a 4-byte column gathered through the permutation
__global__ void __launch_bounds__(64) c_gather4(const uint32_t* col, const uint32_t* perm, uint32_t rows,
                                                uint32_t* sink) {
    const uint32_t stride = gridDim.x * 64;
    uint32_t acc = 0;
    for (uint32_t t = blockIdx.x * 64 + threadIdx.x; t < rows; t += stride) acc ^= col[perm[t]];
    keep(acc, sink);
}

// a 4-byte column read in row order
__global__ void __launch_bounds__(64) c_rows4(const uint32_t* col, uint32_t rows, uint32_t* sink) {
    const uint32_t stride = gridDim.x * 64;
    uint32_t acc = 0;
    for (uint32_t t = blockIdx.x * 64 + threadIdx.x; t < rows; t += stride) acc ^= col[t];
    keep(acc, sink);
}

// 8-byte values read in order (k_chain's base / base1 by visit position)
__global__ void __launch_bounds__(64) c_rows8(const double* col, uint32_t rows, uint32_t* sink) {
    const uint32_t stride = gridDim.x * 64;
    double acc = 0.0;
    for (uint32_t t = blockIdx.x * 64 + threadIdx.x; t < rows; t += stride) acc += col[t];
    keep(acc == 12345.678 ? 0xDEADBEEFu : 0u, sink);
}

// 8-byte values stored in order / scattered through the permutation
__global__ void __launch_bounds__(64) c_store8(double* dst, uint32_t rows) {
    const uint32_t stride = gridDim.x * 64;
    for (uint32_t t = blockIdx.x * 64 + threadIdx.x; t < rows; t += stride) dst[t] = (double)t;
}
__global__ void __launch_bounds__(64) c_scatter8(double* dst, const uint32_t* perm, uint32_t rows) {
    const uint32_t stride = gridDim.x * 64;
    for (uint32_t t = blockIdx.x * 64 + threadIdx.x; t < rows; t += stride) dst[perm[t]] = (double)t;
}

int main(int argc, char** argv) {
    const uint32_t rows = argc > 1 ? (uint32_t)std::strtoul(argv[1], nullptr, 0) : 10000u;
    std::vector<uint32_t> perm(rows);
    std::iota(perm.begin(), perm.end(), 0u);
    std::mt19937 rng(7);
    std::shuffle(perm.begin(), perm.end(), rng);
    const uint32_t n16 = 1u << 22;   // 64 MiB stream
    std::vector<uint32_t> fill((size_t)n16 * 4);
    for (size_t i = 0; i < fill.size(); i++) fill[i] = (uint32_t)(i * 2654435761u) | 1u;
    void *d_stream, *d_tab, *d_col, *d_perm, *d_out, *d_sink;
    CK(hipMalloc(&d_stream, (size_t)n16 * 16));
    CK(hipMalloc(&d_tab, (size_t)rows * 64));
    CK(hipMalloc(&d_col, (size_t)rows * 4));
    CK(hipMalloc(&d_perm, (size_t)rows * 4));
    CK(hipMalloc(&d_out, (size_t)rows * 8));
    CK(hipMalloc(&d_sink, 64));
    CK(hipMemcpy(d_stream, fill.data(), (size_t)n16 * 16, hipMemcpyHostToDevice));
    CK(hipMemcpy(d_tab, fill.data(), (size_t)rows * 64, hipMemcpyHostToDevice));
    CK(hipMemcpy(d_col, fill.data(), (size_t)rows * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(d_perm, perm.data(), (size_t)rows * 4, hipMemcpyHostToDevice));
    auto* sink = (uint32_t*)d_sink;
    auto blocks = [](uint32_t lanes) { return (lanes + 63u) / 64u; };
    // every pattern twice: the first also warms the Infinity Cache (the
    // headline kernels read tables the previous launches just touched)
    for (int rep = 0; rep < 2; rep++) {
        c_stream16<<<4096, 64>>>((const uint4*)d_stream, n16, sink);
        c_rows64<<<blocks(rows), 64>>>((const Rec64*)d_tab, rows, sink);
        c_gather64<false><<<blocks(rows), 64>>>((const Rec64*)d_tab, (const uint32_t*)d_perm, rows, sink);
        c_gather64<true><<<blocks(2 * rows), 64>>>((const Rec64*)d_tab, (const uint32_t*)d_perm, rows, sink);
        c_gather4<<<blocks(rows), 64>>>((const uint32_t*)d_col, (const uint32_t*)d_perm, rows, sink);
        c_rows4<<<blocks(rows), 64>>>((const uint32_t*)d_col, rows, sink);
        c_rows8<<<blocks(rows), 64>>>((const double*)d_out, rows, sink);
        c_store8<<<blocks(rows), 64>>>((double*)d_out, rows);
        c_scatter8<<<blocks(rows), 64>>>((double*)d_out, (const uint32_t*)d_perm, rows);
        CK(hipDeviceSynchronize());
    }
    // unique bytes per pattern (reads / writes)
    std::printf("{\"rows\": %u, \"unique\": {\"c_stream16\": [%llu, 0], \"c_rows64\": [%llu, 0], "
                "\"c_gather64<false>\": [%llu, 0], \"c_gather64<true>\": [%llu, 0], \"c_gather4\": [%llu, 0], "
                "\"c_rows4\": [%llu, 0], \"c_rows8\": [%llu, 0], \"c_store8\": [0, %llu], \"c_scatter8\": [%llu, %llu]}}\n",
                rows, (unsigned long long)n16 * 16, (unsigned long long)rows * 64,
                (unsigned long long)rows * 68, (unsigned long long)rows * 68, (unsigned long long)rows * 8,
                (unsigned long long)rows * 4, (unsigned long long)rows * 8, (unsigned long long)rows * 8,
                (unsigned long long)rows * 4, (unsigned long long)rows * 8);
    return 0;
}
