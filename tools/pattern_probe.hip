// pattern_probe.hip -- speed-of-light probes for the cfg-2 access pattern on MI355X.
//
// What one classifier launch has to move, without any eBPF semantics: per packet a 12-byte
// descriptor (u64 offset + u32 length), a 24-byte header window of its 64-byte packet, an 8-byte
// r0 and a 1-byte status; per vCPU one 32-byte counter row read and written.  The probes run that
// pattern (and a plain streaming read of the same bytes) over NB rotating batches so no batch is
// served from the 256 MiB Infinity Cache, and report microseconds per launch (HIP events).
//
//   hipcc --offload-arch=gfx950 -O3 -o pattern_probe tools/pattern_probe.hip && ./pattern_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                                  \
    do {                                                                                       \
        hipError_t e_ = (x);                                                                   \
        if (e_ != hipSuccess) {                                                                \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));         \
            exit(1);                                                                           \
        }                                                                                      \
    } while (0)

struct Batch {
    uint8_t *pkt;
    uint64_t *off;
    uint32_t *len;
    uint64_t *r0;
    uint8_t *st;
};

// plain streaming read of `bytes` (16-byte loads, grid-stride), one word written per block
__global__ void stream_read(const uint4 *p, size_t n16, uint64_t *sink) {
    uint64_t acc = 0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n16; i += (size_t)gridDim.x * blockDim.x) {
        const uint4 v = p[i];
        acc ^= v.x ^ v.y ^ v.z ^ v.w;
    }
    if (acc == 0x1234567) sink[blockIdx.x] = acc;
}

// the classifier's pattern: lane g runs packets g, g + V, g + 2V, ... (interleaved schedule) or
// g*per .. (chunked); per packet descriptor -> header window -> r0 / status; counter row in
// registers for the launch (the JIT's lane value cache).  DEPTH > 1 issues the next packets'
// descriptors and windows early (software pipelining across a lane's packets).
template <int DEPTH>
__global__ __launch_bounds__(256) void classify_pattern(Batch b, uint32_t n, uint32_t V, int chunked,
                                                        uint64_t *rows) {
    const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= V) return;
    const uint32_t per = (n + V - 1) / V;
    uint64_t c0 = rows[4 * (size_t)g], c1 = rows[4 * (size_t)g + 1], c2 = rows[4 * (size_t)g + 2],
             c3 = rows[4 * (size_t)g + 3];
    auto idx = [&](uint32_t j) -> uint32_t { return chunked ? g * per + j : j * V + g; };
    uint64_t w0[DEPTH], w1[DEPTH], w2[DEPTH];
    uint32_t ln[DEPTH];
    auto issue = [&](uint32_t j, int s) {
        const uint32_t i = idx(j);
        if (j < per && i < n) {
            const uint64_t o = b.off[i];
            ln[s] = b.len[i];
            const uint64_t *h = (const uint64_t *)(b.pkt + o + 8);
            w0[s] = h[0];
            w1[s] = h[1];
            w2[s] = h[2];
        }
    };
#pragma unroll
    for (int s = 0; s < DEPTH; s++) issue(s, s);
    for (uint32_t j = 0; j < per; j++) {
        const int s = j % DEPTH;
        const uint32_t i = idx(j);
        if (i >= n) break;
        const uint64_t a = w0[s], c = w1[s], d = w2[s];
        const uint32_t L = ln[s];
        if (DEPTH > 1) issue(j + DEPTH, s);   // refill this stage (values above already taken)
        uint64_t h = ((c >> 48) | (d << 16)) ^ (d >> 16);
        h ^= h >> 16;
        h = (h * 0x9e3779b1ull) ^ (c >> 24);
        h ^= h >> 13;
        const uint32_t v = (L >= 34 && (uint16_t)(a >> 32) == 8) ? ((h & 3) ? 2u : 1u) : 2u;
        c0 += v == 0;
        c1 += v == 1;
        c2 += v == 2;
        c3 += v == 3;
        __builtin_nontemporal_store((uint64_t)v, b.r0 + i);
        __builtin_nontemporal_store((uint8_t)0, b.st + i);
        if (DEPTH == 1 && j + 1 < per) issue(j + 1, 0);
    }
    rows[4 * (size_t)g] = c0;
    rows[4 * (size_t)g + 1] = c1;
    rows[4 * (size_t)g + 2] = c2;
    rows[4 * (size_t)g + 3] = c3;
}

template <class F>
static float time_us(F launch, int reps) {
    hipEvent_t a, z;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&z));
    for (int k = 0; k < 5; k++) launch(k);
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(a));
    for (int k = 0; k < reps; k++) launch(k);
    CK(hipEventRecord(z));
    CK(hipEventSynchronize(z));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, a, z));
    return ms * 1e3f / reps;
}

int main(int argc, char **argv) {
    const uint32_t n = 1u << 20, V = argc > 1 ? (uint32_t)atoi(argv[1]) : (1u << 18);
    const int NB = 5, reps = 50;
    std::vector<Batch> bs(NB);
    std::vector<uint64_t> off(n);
    std::vector<uint32_t> len(n, 64);
    for (uint32_t i = 0; i < n; i++) off[i] = 64ull * i;
    std::vector<uint8_t> pk(64ull * n);
    for (size_t i = 0; i < pk.size(); i++) pk[i] = (uint8_t)(i * 2654435761u >> 13);
    for (uint32_t i = 0; i < n; i++) { pk[64ull * i + 12] = 8; pk[64ull * i + 13] = 0; }
    for (auto &b : bs) {
        CK(hipMalloc(&b.pkt, 64ull * n));
        CK(hipMalloc(&b.off, 8ull * n));
        CK(hipMalloc(&b.len, 4ull * n));
        CK(hipMalloc(&b.r0, 8ull * n));
        CK(hipMalloc(&b.st, n));
        CK(hipMemcpy(b.pkt, pk.data(), pk.size(), hipMemcpyHostToDevice));
        CK(hipMemcpy(b.off, off.data(), 8ull * n, hipMemcpyHostToDevice));
        CK(hipMemcpy(b.len, len.data(), 4ull * n, hipMemcpyHostToDevice));
    }
    uint64_t *rows, *sink;
    CK(hipMalloc(&rows, 32ull * V));
    CK(hipMemset(rows, 0, 32ull * V));
    CK(hipMalloc(&sink, 8 << 20));
    const double alg = 64.0 * n + 16.0 * n + 2.0 * 32 * V;   // SURVEY 8(d) bytes per launch
    const double moved = 64.0 * n + 12.0 * n + 9.0 * n + 2.0 * 32 * V;
    printf("n %u V %u, %d rotating batches; algorithmic %.1f MB, moved %.1f MB per launch\n", n, V, NB, alg / 1e6,
           moved / 1e6);
    const float t_stream = time_us([&](int k) {
        stream_read<<<8192, 256>>>((const uint4 *)bs[k % NB].pkt, 64ull * n / 16, sink);
    }, reps);
    printf("stream_read 64 MiB packets: %.2f us  %.2f TB/s\n", t_stream, 64.0 * n / t_stream / 1e6);
    const uint32_t blocks = (V + 255) / 256;
    for (int chunked = 0; chunked < 2; chunked++) {
        float t1 = time_us([&](int k) { classify_pattern<1><<<blocks, 256>>>(bs[k % NB], n, V, chunked, rows); }, reps);
        float t2 = time_us([&](int k) { classify_pattern<2><<<blocks, 256>>>(bs[k % NB], n, V, chunked, rows); }, reps);
        float t4 = time_us([&](int k) { classify_pattern<4><<<blocks, 256>>>(bs[k % NB], n, V, chunked, rows); }, reps);
        printf("%s: depth1 %.2f us (%.2f TB/s alg)  depth2 %.2f us  depth4 %.2f us (%.2f TB/s alg)\n",
               chunked ? "chunked" : "interleaved", t1, alg / t1 / 1e6, t2, t4, alg / t4 / 1e6);
    }
    return 0;
}
