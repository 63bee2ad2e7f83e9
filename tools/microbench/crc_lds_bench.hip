// CRC32-IEEE throughput of segment-parallel LDS table variants (dev tool, not
// product code).  Each wave stages 64 segments of 36 bytes (2304 B) from HBM
// into LDS with LDS-DMA, then every lane computes raw(0, segment) -- the CRC
// register after its 36 bytes from state 0 -- with no serial chain:
//   nib : XOR over the 72 nibbles of NT[p][h][nibble] (16-entry tables, which
//         occupy 16 distinct banks: conflict-free whatever the data)
//   byte: XOR over the 36 bytes of T[p][byte] (256-entry tables, 36 KiB)
//   none: the staging and reads only
// and checks the per-segment values of the first segments against the host.
// usage: crc_lds_bench [GiB]
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define CK(x)                                                                              \
    do {                                                                                   \
        hipError_t e_ = (x);                                                               \
        if (e_ != hipSuccess) {                                                            \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            exit(1);                                                                       \
        }                                                                                  \
    } while (0)

constexpr int kSeg = 36;               // bytes per segment
constexpr int kGroup = 64 * kSeg;      // bytes per wave round
constexpr int kWaves = 4;

__constant__ uint32_t c_nib[kSeg * 2 * 16];
__constant__ uint32_t c_byte[kSeg * 256];

template <int MODE>
__global__ __launch_bounds__(256) void crc_kernel(const uint8_t *__restrict__ buf, uint64_t nseg,
                                                  uint32_t *__restrict__ out, uint32_t *__restrict__ first) {
    __shared__ uint32_t tab[MODE == 1 ? kSeg * 256 : kSeg * 32];
    __shared__ __attribute__((aligned(16))) uint8_t stage[kWaves][kGroup + 64];
    const uint32_t tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    if (MODE == 1)
        for (uint32_t i = tid; i < kSeg * 256; i += 256) tab[i] = c_byte[i];
    else
        for (uint32_t i = tid; i < kSeg * 32; i += 256) tab[i] = c_nib[i];
    __syncthreads();
    uint8_t *st = stage[wave];
    const uint64_t ngroups = nseg / 64;
    uint32_t acc = 0;
    for (uint64_t g = (uint64_t)blockIdx.x * kWaves + wave; g < ngroups; g += (uint64_t)gridDim.x * kWaves) {
        const uint8_t *src = buf + g * kGroup;
#pragma unroll
        for (int k = 0; k < 3; k++) {
            const uint32_t c = k * 64 + lane;
            if (c < kGroup / 16)
                __builtin_amdgcn_global_load_lds((const void *)(src + 16 * c),
                                                 (__attribute__((address_space(3))) void *)(st + k * 1024), 16, 0, 0);
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        const uint32_t *w = reinterpret_cast<const uint32_t *>(st) + 9 * lane;
        uint32_t x[9];
#pragma unroll
        for (int i = 0; i < 9; i++) x[i] = w[i];
        uint32_t r = 0;
        if (MODE == 0) {
#pragma unroll
            for (int i = 0; i < 9; i++) {
                const uint32_t lo = (x[i] & 0x0F0F0F0Fu) << 2, hi = (x[i] >> 2) & 0x3C3C3C3Cu;
#pragma unroll
                for (int b = 0; b < 4; b++) {
                    const int p = kSeg - 1 - (4 * i + b);
                    const uint32_t il = (lo >> (8 * b)) & 0xFF, ih = (hi >> (8 * b)) & 0xFF;
                    r ^= tab[(p * 2 + 0) * 16 + (il >> 2)] ^ tab[(p * 2 + 1) * 16 + (ih >> 2)];
                }
            }
        } else if (MODE == 1) {
#pragma unroll
            for (int i = 0; i < 9; i++)
#pragma unroll
                for (int b = 0; b < 4; b++) {
                    const int p = kSeg - 1 - (4 * i + b);
                    r ^= tab[p * 256 + ((x[i] >> (8 * b)) & 0xFF)];
                }
        } else {
#pragma unroll
            for (int i = 0; i < 9; i++) r ^= x[i];
        }
        if (g < 4) first[g * 64 + lane] = r;
        acc = (acc << 1 | acc >> 31) ^ r;
        // the next DMA may overwrite the staging area: every lane has read it
        __builtin_amdgcn_wave_barrier();
    }
    out[blockIdx.x * 256 + tid] = acc;
}

static uint32_t host_tab[256];
static uint32_t raw_step(uint32_t c, uint8_t b) { return host_tab[(c ^ b) & 0xFF] ^ (c >> 8); }

int main(int argc, char **argv) {
    const double gib = argc > 1 ? atof(argv[1]) : 2.0;
    for (uint32_t i = 0; i < 256; i++) {
        uint32_t c = i;
        for (int k = 0; k < 8; k++) c = (c & 1) ? 0xEDB88320u ^ (c >> 1) : c >> 1;
        host_tab[i] = c;
    }
    // T[p][b] = raw(0, b followed by p zero bytes)
    std::vector<uint32_t> T(kSeg * 256), N(kSeg * 32);
    for (int b = 0; b < 256; b++) {
        uint32_t c = raw_step(0, (uint8_t)b);
        for (int p = 0; p < kSeg; p++) {
            T[p * 256 + b] = c;
            c = raw_step(c, 0);
        }
    }
    for (int p = 0; p < kSeg; p++)
        for (int v = 0; v < 16; v++) {
            N[(p * 2 + 0) * 16 + v] = T[p * 256 + v];
            N[(p * 2 + 1) * 16 + v] = T[p * 256 + (v << 4)];
        }
    CK(hipMemcpyToSymbol(HIP_SYMBOL(c_nib), N.data(), N.size() * 4));
    CK(hipMemcpyToSymbol(HIP_SYMBOL(c_byte), T.data(), T.size() * 4));
    const uint64_t bytes = ((uint64_t)(gib * (1ull << 30)) / kGroup) * kGroup;
    const uint64_t nseg = bytes / kSeg;
    std::vector<uint8_t> h(1 << 20);
    uint64_t s = 88172645463325252ull;
    for (auto &v : h) { s ^= s << 13; s ^= s >> 7; s ^= s << 17; v = (uint8_t)s; }
    uint8_t *d;
    CK(hipMalloc(&d, bytes + 4096));
    for (uint64_t o = 0; o < bytes; o += h.size()) CK(hipMemcpy(d + o, h.data(), std::min<uint64_t>(h.size(), bytes - o), hipMemcpyHostToDevice));
    int cus = 0;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    uint32_t *out, *first;
    const int maxblocks = cus * 8;
    CK(hipMalloc(&out, (size_t)maxblocks * 256 * 4));
    CK(hipMalloc(&first, 256 * 4));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    // expected first 256 segments
    std::vector<uint32_t> want(256);
    for (int g = 0; g < 256; g++) {
        uint32_t c = 0;
        for (int i = 0; i < kSeg; i++) c = raw_step(c, h[g * kSeg + i]);
        want[g] = c;
    }
    const char *names[3] = {"nib", "byte", "none"};
    for (int mode = 0; mode < 3; mode++) {
        for (int per = 2; per <= 8; per *= 2) {
            const int blocks = cus * per;
            float best = 1e30f;
            for (int it = 0; it < 6; it++) {
                CK(hipEventRecord(e0, 0));
                if (mode == 0) hipLaunchKernelGGL(crc_kernel<0>, dim3(blocks), dim3(256), 0, 0, d, nseg, out, first);
                if (mode == 1) hipLaunchKernelGGL(crc_kernel<1>, dim3(blocks), dim3(256), 0, 0, d, nseg, out, first);
                if (mode == 2) hipLaunchKernelGGL(crc_kernel<2>, dim3(blocks), dim3(256), 0, 0, d, nseg, out, first);
                CK(hipGetLastError());
                CK(hipEventRecord(e1, 0));
                CK(hipEventSynchronize(e1));
                float ms = 0;
                CK(hipEventElapsedTime(&ms, e0, e1));
                if (it > 0 && ms < best) best = ms;
            }
            std::vector<uint32_t> got(256);
            CK(hipMemcpy(got.data(), first, 256 * 4, hipMemcpyDeviceToHost));
            int bad = 0;
            if (mode < 2)
                for (int g = 0; g < 256; g++) bad += got[g] != want[g];
            printf("%-5s blocks/CU %d: %.3f ms  %.0f GB/s  (%.3f of 8 TB/s)  check %s\n", names[mode], per, best,
                   bytes / (best * 1e-3) / 1e9, bytes / (best * 1e-3) / 8e12, bad ? "FAIL" : "ok");
        }
    }
    return 0;
}
