// Cross-queue hand-off microbenchmark (gfx950): what the pipelined numpy-MT
// step pays between consecutive play launches for each way of ordering the
// play kernel (stream A, one 256-thread block per CU, ~120 KB LDS, a long
// latency-bound body) after a concurrent "twist" kernel (stream S, 16 384
// small blocks, memory-bound) and the twist after the play launch before.
//
//   serial   A: play(i); twist(i+1)                       (one stream)
//   events   A: wait(ev_twist); record(ev_play); play      S: wait(ev_play); twist; record(ev_twist)
//            (the library's SN_OPT_PIPELINE schedule through round 3)
//   flags    A: play only -- each play wave polls its 64 games' generation
//            words (sc1) that the twist waves store after their sc1 payload
//            stores drained; S: hipStreamWaitValue32 on a counter the play
//            blocks add to after their sc1 stores drained, then twist
//   alone    A: play only, no twist (the floor)
//
// Every play lane checks every payload word it reads against the generation
// (counts stale words) and every spin is bounded (a timeout counts, no hang).
// Build: hipcc --offload-arch=gfx950 -O3 -o /tmp/queue_gap tools/queue_gap.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                              \
    do {                                                                                   \
        hipError_t e_ = (x);                                                               \
        if (e_ != hipSuccess) {                                                            \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            exit(1);                                                                       \
        }                                                                                  \
    } while (0)

constexpr int B = 65536;        // games
constexpr int PAY = 16;         // payload dwords per game per launch (ring bytes stand-in)
constexpr int TW = 768;         // dwords of "MT state" per game the twist reads+writes (~196 MB of traffic per launch)
constexpr int PLAY_LDS = 120 * 1024;

struct Shared {
    uint32_t* gen;    // [B] generation of the payload the twist wrote last
    uint32_t* pay;    // [B][PAY] payload
    uint32_t* mt;     // [B][TW]
    uint32_t* cnt;    // signal memory: play blocks finished (monotonic)
    uint32_t* stale;  // [2] stale words seen, spin timeouts
    uint32_t* pabs;   // [B] play output the twist reads
};

__device__ __forceinline__ uint32_t ld_sc1(const uint32_t* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_sc1(uint32_t* p, uint32_t v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// play: one game per lane, 64 games per wave, 4 waves per block
__global__ __launch_bounds__(256) void k_play(Shared s, uint32_t gen, int poll, int busy_ticks) {
    extern __shared__ uint32_t lds[];
    const int g = blockIdx.x * 256 + threadIdx.x;
    if (poll) {
        // bounded poll of this lane's game generation, wave-uniform exit
        uint64_t t0 = wall_clock64();
        bool ok = false;
        while (true) {
            ok = ld_sc1(&s.gen[g]) >= gen;
            if (__all(ok)) break;
            if (wall_clock64() - t0 > 10000000ull) {  // 100 ms at 100 MHz
                if (!ok) atomicAdd(&s.stale[1], 1u);
                break;
            }
            __builtin_amdgcn_s_sleep(2);
        }
        __atomic_signal_fence(__ATOMIC_SEQ_CST);
    }
    uint32_t acc = 0, bad = 0;
#pragma unroll
    for (int k = 0; k < PAY; k++) {
        const size_t at = ((size_t)(gen & 1u) * PAY + k) * B + g;  // double-buffered by launch parity
        const uint32_t v = poll ? ld_sc1(&s.pay[at]) : s.pay[at];
        bad += (v != gen * 131u + (uint32_t)g + (uint32_t)k) ? 1u : 0u;
        acc += v;
    }
    lds[threadIdx.x] = acc;
    // latency-bound body stand-in
    const uint64_t t0 = wall_clock64();
    uint32_t x = acc;
    while (wall_clock64() - t0 < (uint64_t)busy_ticks) {
#pragma unroll
        for (int j = 0; j < 16; j++) x = x * 1664525u + 1013904223u;
    }
    lds[threadIdx.x + 256] = x;
    if (poll && bad) atomicAdd(&s.stale[0], bad);
    st_sc1(&s.pabs[g], x | 1u);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) __hip_atomic_fetch_add(s.cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// twist: one wave per game
__global__ __launch_bounds__(256) void k_twist(Shared s, uint32_t gen) {
    const int g = blockIdx.x * 4 + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    uint32_t* m = s.mt + (size_t)g * TW;
    const uint32_t pa = s.pabs[g];
    uint32_t v[TW / 64];
#pragma unroll
    for (int k = 0; k < TW / 64; k++) v[k] = m[k * 64 + lane];
#pragma unroll
    for (int k = 0; k < TW / 64; k++) m[k * 64 + lane] = v[k] * 69069u + pa;
    if (lane < PAY) st_sc1(&s.pay[((size_t)(gen & 1u) * PAY + lane) * B + g], gen * 131u + (uint32_t)g + (uint32_t)lane);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (lane == 0) st_sc1(&s.gen[g], gen);
}

int main(int argc, char** argv) {
    const int iters = argc > 1 ? atoi(argv[1]) : 200;
    const int busy_us = argc > 2 ? atoi(argv[2]) : 62;
    int can_wait = 0;
    CK(hipDeviceGetAttribute(&can_wait, hipDeviceAttributeCanUseStreamWaitValue, 0));
    Shared s;
    CK(hipMalloc(&s.gen, B * 4));
    CK(hipMalloc(&s.pay, (size_t)2 * B * PAY * 4));
    CK(hipMalloc(&s.mt, (size_t)B * TW * 4));
    CK(hipMalloc(&s.stale, 8));
    CK(hipMalloc(&s.pabs, B * 4));
    CK(hipExtMallocWithFlags((void**)&s.cnt, 8, hipMallocSignalMemory));
    CK(hipMemset(s.mt, 0, (size_t)B * TW * 4));
    CK(hipFuncSetAttribute((const void*)k_play, hipFuncAttributeMaxDynamicSharedMemorySize, PLAY_LDS));
    hipStream_t A, S;
    CK(hipStreamCreateWithFlags(&A, hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&S, hipStreamNonBlocking));
    hipEvent_t evp, evt, t0, t1;
    CK(hipEventCreateWithFlags(&evp, hipEventDisableTiming | hipEventDisableSystemFence));
    CK(hipEventCreateWithFlags(&evt, hipEventDisableTiming | hipEventDisableSystemFence));
    CK(hipEventCreate(&t0));
    CK(hipEventCreate(&t1));
    const int busy = busy_us * 100;  // wall_clock64 ticks at 100 MHz
    printf("{\"can_use_stream_wait_value\": %d, \"iters\": %d, \"busy_us\": %d}\n", can_wait, iters, busy_us);
    const char* names[] = {"alone", "serial", "events", "flags"};
    for (int rep = 0; rep < 2; rep++)
        for (int mode = 0; mode < 4; mode++) {
            if (mode == 3 && !can_wait) continue;
            CK(hipMemset(s.gen, 0, B * 4));
            CK(hipMemset(s.stale, 0, 8));
            CK(hipMemset(s.cnt, 0, 4));
            CK(hipDeviceSynchronize());
            // launch 1's payload, synchronously
            hipLaunchKernelGGL(k_twist, dim3(B / 4), dim3(256), 0, A, s, 1u);
            CK(hipStreamSynchronize(A));
            CK(hipEventRecord(evt, A));
            uint32_t nb = B / 256;
            CK(hipEventRecord(t0, A));
            for (int i = 1; i <= iters; i++) {
                const uint32_t gen = (uint32_t)i;
                if (mode == 0) {
                    hipLaunchKernelGGL(k_play, dim3(B / 256), dim3(256), PLAY_LDS, A, s, gen, 0, busy);
                } else if (mode == 1) {
                    hipLaunchKernelGGL(k_play, dim3(B / 256), dim3(256), PLAY_LDS, A, s, gen, 0, busy);
                    hipLaunchKernelGGL(k_twist, dim3(B / 4), dim3(256), 0, A, s, gen + 1);
                } else if (mode == 2) {
                    CK(hipStreamWaitEvent(A, evt, 0));
                    CK(hipEventRecord(evp, A));
                    hipLaunchKernelGGL(k_play, dim3(B / 256), dim3(256), PLAY_LDS, A, s, gen, 0, busy);
                    CK(hipStreamWaitEvent(S, evp, 0));
                    hipLaunchKernelGGL(k_twist, dim3(B / 4), dim3(256), 0, S, s, gen + 1);
                    CK(hipEventRecord(evt, S));
                } else {
                    hipLaunchKernelGGL(k_play, dim3(B / 256), dim3(256), PLAY_LDS, A, s, gen, 1, busy);
                    // twist(i+1) after play(i-1): the play blocks' counter
                    CK(hipStreamWaitValue32(S, s.cnt, (uint32_t)(i - 1) * nb, hipStreamWaitValueGte, 0xFFFFFFFFu));
                    hipLaunchKernelGGL(k_twist, dim3(B / 4), dim3(256), 0, S, s, gen + 1);
                }
            }
            CK(hipEventRecord(t1, A));
            CK(hipDeviceSynchronize());
            float ms = 0;
            CK(hipEventElapsedTime(&ms, t0, t1));
            uint32_t st[2];
            CK(hipMemcpy(st, s.stale, 8, hipMemcpyDeviceToHost));
            printf("{\"mode\": \"%s\", \"rep\": %d, \"us_per_iter\": %.2f, \"stale_words\": %u, \"timeouts\": %u}\n",
                   names[mode], rep, ms * 1e3 / iters, st[0], st[1]);
            fflush(stdout);
        }
    return 0;
}
