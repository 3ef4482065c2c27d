// tools/xcd_visibility_probe.hip -- the precondition of round 2's stale-tile defect
// (not product).
//
// Round 2's drop-in read a multi-tile result in host memory back stale on 4 of 6 boxes:
// the op's workgroups ran on several XCDs, and the completion signal -- one lane that
// ran __threadfence_system() and stored a flag -- wrote back only its own XCD's L2.
// This replays exactly that protocol (no release in the writing kernel) for each kind
// of host memory the library or a caller may hand the kernels, and counts stale bytes
// the host reads right after the flag:
//   mapped_coherent   hipHostMallocMapped | hipHostMallocCoherent (the zero-copy staging)
//   coherent          hipHostMallocCoherent
//   default           hipHostMallocDefault (torch pin_memory)
//   noncoherent       hipHostMallocNonCoherent
// and the same with the fixed protocol (every writing wave ends with a system-scope
// release and s_waitcnt vmcnt(0), the library's kSysRel epilogue) as the control.
// It also prints what identifies the box's memory mapping: kernel release, amdgpu
// driver version, and the amdgpu module parameters that set memory types.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/xcd_visibility_probe.hip -o tools/xcd_visibility_probe.bin
#include <hip/hip_runtime.h>

#include <sys/utsname.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>

#define CK(x)                                                              \
    do {                                                                   \
        hipError_t ck_ = (x);                                              \
        if (ck_ != hipSuccess) {                                           \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(ck_));       \
            exit(1);                                                       \
        }                                                                  \
    } while (0)

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
#define GL __attribute__((address_space(1)))

// dst[i] ^= 0x5A per 16-byte chunk: one 4 KiB tile per 256-lane workgroup, as the
// drop-in's launch over a host destination.  kRel: the kSysRel epilogue.
template <bool kRel>
__global__ __launch_bounds__(256) void k_write(uint8_t *dst) {
    const uint64_t off = (uint64_t)blockIdx.x * 4096 + threadIdx.x * 16;
    u32x4 v = *(const GL u32x4 *)((uintptr_t)dst + off);
    v ^= (u32x4){0x5A5A5A5Au, 0x5A5A5A5Au, 0x5A5A5A5Au, 0x5A5A5A5Au};
    __builtin_nontemporal_store(v, (GL u32x4 *)((uintptr_t)dst + off));
    if constexpr (kRel) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
        __asm__ volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
}

// Round 2's completion signal: one lane, its own fence, a system-scope flag store.
__global__ void k_signal(uint32_t *flag, uint32_t v) {
    __threadfence_system();
    __hip_atomic_store(flag, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

static std::string slurp(const char *path) {
    FILE *f = fopen(path, "r");
    if (!f) return "n/a";
    char buf[256] = "";
    size_t n = fread(buf, 1, sizeof buf - 1, f);
    fclose(f);
    buf[n] = 0;
    while (n && (buf[n - 1] == '\n' || buf[n - 1] == ' ')) buf[--n] = 0;
    return buf;
}

int main(int argc, char **argv) {
    const int tiles = argc > 1 ? atoi(argv[1]) : 64;
    const int reps = argc > 2 ? atoi(argv[2]) : 200;
    struct utsname u;
    uname(&u);
    printf("{\"box\": {\"kernel\": \"%s\", \"amdgpu_version\": \"%s\", \"mtype_local\": \"%s\", "
           "\"amdgpu_noretry\": \"%s\", \"amdgpu_vm_update_mode\": \"%s\", \"hsa_xnack\": \"%s\"}}\n",
           u.release, slurp("/sys/module/amdgpu/version").c_str(),
           slurp("/sys/module/amdgpu/parameters/mtype_local").c_str(),
           slurp("/sys/module/amdgpu/parameters/noretry").c_str(),
           slurp("/sys/module/amdgpu/parameters/vm_update_mode").c_str(),
           getenv("HSA_XNACK") ? getenv("HSA_XNACK") : "unset");
    const size_t n = (size_t)tiles * 4096;
    uint32_t *flag;
    CK(hipHostMalloc((void **)&flag, 64, hipHostMallocMapped | hipHostMallocCoherent));
    uint32_t *flag_dev;
    CK(hipHostGetDevicePointer((void **)&flag_dev, flag, 0));
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    struct Kind {
        const char *name;
        unsigned flags;
    } kinds[] = {{"mapped_coherent", hipHostMallocMapped | hipHostMallocCoherent},
                 {"coherent", hipHostMallocCoherent},
                 {"default", hipHostMallocDefault},
                 {"noncoherent", hipHostMallocNonCoherent}};
    uint32_t seq = 0;
    for (const Kind &k : kinds) {
        uint8_t *h;
        CK(hipHostMalloc((void **)&h, n, k.flags));
        uint8_t *d;
        CK(hipHostGetDevicePointer((void **)&d, h, 0));
        for (int rel = 0; rel < 2; ++rel) {
            long stale_bytes = 0, stale_calls = 0, stale_tiles_max = 0, slow = 0;
            for (int r = 0; r < reps; ++r) {
                const uint8_t base = (uint8_t)(r * 37 + 11);
                memset(h, base, n);
                __atomic_thread_fence(__ATOMIC_SEQ_CST);
                if (rel) k_write<true><<<tiles, 256, 0, s>>>(d);
                else k_write<false><<<tiles, 256, 0, s>>>(d);
                const uint32_t v = ++seq;
                k_signal<<<1, 1, 0, s>>>(flag_dev, v);
                const auto t0 = std::chrono::steady_clock::now();
                while (__atomic_load_n(flag, __ATOMIC_ACQUIRE) != v) {
                    if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(2)) {
                        ++slow;
                        CK(hipStreamSynchronize(s));
                        break;
                    }
                }
                const uint8_t want = base ^ 0x5A;
                long bad = 0, bad_tiles = 0;
                for (int t = 0; t < tiles; ++t) {
                    long bt = 0;
                    for (size_t i = 0; i < 4096; ++i) bt += h[(size_t)t * 4096 + i] != want;
                    bad += bt;
                    bad_tiles += bt != 0;
                }
                CK(hipStreamSynchronize(s));
                stale_bytes += bad;
                stale_calls += bad != 0;
                if (bad_tiles > stale_tiles_max) stale_tiles_max = bad_tiles;
            }
            printf("{\"memory\": \"%s\", \"writer_release\": %s, \"tiles\": %d, \"calls\": %d, "
                   "\"stale_calls\": %ld, \"stale_bytes\": %ld, \"max_stale_tiles\": %ld, \"flag_timeouts\": %ld}\n",
                   k.name, rel ? "true" : "false", tiles, reps, stale_calls, stale_bytes, stale_tiles_max, slow);
            fflush(stdout);
        }
        CK(hipHostFree(h));
    }
    CK(hipStreamDestroy(s));
    CK(hipHostFree(flag));
    return 0;
}
