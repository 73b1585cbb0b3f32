// NUMA placement of the host side of each GPU (one host thread
// + stream + NUMA-local pinned buffers per GPU). helyim itself is CPU-only and
// NUMA-unaware; the GPU path adds PCIe and host-DRAM traffic per GPU, so every
// pinned buffer this library allocates lives on the NUMA node of the GPU that
// reads it over PCIe, and a caller (one process or thread per GPU) can bind its
// CPUs to that node too.
//
// Node of a GPU: sysfs numa_node of its PCI function (hipDeviceGetPCIBusId).
// Placement: the allocating thread's memory policy is set to MPOL_PREFERRED on
// that node around hipHostMalloc(hipHostMallocNumaUser), which makes the
// runtime follow the thread's policy when it backs the pinned range, then
// restored. One host batch split over several GPUs (hec_host_alloc_multi) gets
// each stripe range's pages on its own GPU's node (mbind).
// Raw syscalls, so libhec needs no libnuma.
#include <sched.h>
#include <sys/mman.h>
#include <sys/syscall.h>
#include <unistd.h>

#include <cctype>
#include <cstdlib>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <map>
#include <string>
#include <vector>

#include "hec_internal.hpp"

namespace hec {
namespace {

constexpr int kMpolDefault = 0;
constexpr int kMpolPreferred = 1;
constexpr unsigned kMaxNodes = 1024;
constexpr size_t kMaskWords = kMaxNodes / (8 * sizeof(unsigned long));

std::string read_line(const std::string& path) {
    std::ifstream f(path);
    std::string s;
    if (f) std::getline(f, s);
    return s;
}

int online_nodes() {
    // "0" or "0-1" or "0,2-3": count nodes
    const std::string s = read_line("/sys/devices/system/node/online");
    if (s.empty()) return 1;
    int n = 0;
    size_t i = 0;
    while (i < s.size()) {
        int a = 0, b;
        if (sscanf(s.c_str() + i, "%d-%d", &a, &b) == 2) n += b - a + 1;
        else n += 1;
        size_t j = s.find(',', i);
        if (j == std::string::npos) break;
        i = j + 1;
    }
    return n > 0 ? n : 1;
}

// CPU list syntax ("0-15,128-143") -> ids
std::vector<int> parse_cpulist(const std::string& s) {
    std::vector<int> out;
    size_t i = 0;
    while (i < s.size()) {
        int a, b;
        if (sscanf(s.c_str() + i, "%d-%d", &a, &b) == 2) {
            for (int c = a; c <= b; ++c) out.push_back(c);
        } else if (sscanf(s.c_str() + i, "%d", &a) == 1) {
            out.push_back(a);
        }
        size_t j = s.find(',', i);
        if (j == std::string::npos) break;
        i = j + 1;
    }
    return out;
}

}  // namespace

int device_numa_node(int device, int* node) {
    *node = -1;
    char bus[64] = {0};
    HEC_HIP(hipDeviceGetPCIBusId(bus, sizeof(bus), device));
    std::string id(bus);
    for (auto& ch : id) ch = char(std::tolower(static_cast<unsigned char>(ch)));
    const std::string s = read_line("/sys/bus/pci/devices/" + id + "/numa_node");
    if (!s.empty()) *node = std::atoi(s.c_str());
    return HEC_OK;
}

// Test hook: HEC_TEST_NUMA_BIND_FAIL=1 makes every NUMA-placed allocation
// attempt fail after it ran, as if the node could not back it, so the
// fallback below runs on any machine (tests/test_gpu_numa.py).
static bool bind_failure_forced() {
    static const bool forced = [] {
        const char* v = std::getenv("HEC_TEST_NUMA_BIND_FAIL");
        return v && v[0] == '1';
    }();
    return forced;
}

// Pinned host memory on the current device's NUMA node (plain hipHostMalloc
// when the node is unknown or the machine has one node). The allocating
// thread's policy is MPOL_PREFERRED on the node around
// hipHostMalloc(hipHostMallocNumaUser): placement is a speed preference,
// never a requirement, so a short node spills to the others page by page
// (MPOL_BIND would wake the constrained OOM killer during pinning instead of
// failing). Should the placed attempt still fail, the allocation is retried
// under the default policy instead of failing.
int pinned_alloc(void** p, size_t bytes) {
    *p = nullptr;
    int dev, node = -1, rc;
    if ((rc = current_device(&dev))) return rc;
    if ((rc = device_numa_node(dev, &node))) return rc;
    const unsigned flags = hipHostMallocPortable;  // every device may code it zero-copy (_multi ranges)
    if (node < 0 || node >= int(kMaxNodes) || online_nodes() < 2) {
        HEC_HIP(hipHostMalloc(p, bytes, flags));
        return HEC_OK;
    }
    unsigned long old_mask[kMaskWords] = {0};
    int old_mode = kMpolDefault;
    const bool saved = syscall(SYS_get_mempolicy, &old_mode, old_mask, kMaxNodes, nullptr, 0) == 0;
    unsigned long mask[kMaskWords] = {0};
    mask[node / (8 * sizeof(unsigned long))] = 1ul << (node % (8 * sizeof(unsigned long)));
    const bool placed = syscall(SYS_set_mempolicy, kMpolPreferred, mask, kMaxNodes) == 0;
    hipError_t e = hipHostMalloc(p, bytes, placed ? (flags | hipHostMallocNumaUser) : flags);
    if (placed) {
        if (saved) (void)syscall(SYS_set_mempolicy, old_mode, old_mode == kMpolDefault ? nullptr : old_mask,
                                 kMaxNodes);
        else (void)syscall(SYS_set_mempolicy, kMpolDefault, nullptr, 0);
    }
    if (e == hipSuccess && bind_failure_forced()) {  // test hook: as if the placed attempt failed
        (void)hipHostFree(*p);
        e = hipErrorOutOfMemory;
    }
    if (e == hipSuccess) return HEC_OK;
    (void)hipGetLastError();
    *p = nullptr;
    e = hipHostMalloc(p, bytes, flags);  // any node: placement is speed only
    if (e != hipSuccess) return hip_fail(e, "hipHostMalloc (pinned, after the NUMA-local attempt failed)");
    return HEC_OK;
}

// ---------------------------------------------------------------------------
// Host batches placed per stripe range (hec_host_alloc_multi): anonymous
// memory, each range's pages preferred on its device's node (mbind before the
// first touch), then pinned and mapped for every device (hipHostRegister).
// hec_host_free recognises these by address.
// ---------------------------------------------------------------------------
std::mutex& placed_mu() {
    static std::mutex* m = new std::mutex();
    return *m;
}
std::map<void*, size_t>& placed_allocs() {
    static auto* m = new std::map<void*, size_t>();  // process lifetime
    return *m;
}

// Test hook: HEC_TEST_RANGE_NODES="a,b,..." gives range r node r-th entry
// instead of its device's node (a one-GPU box lists one device twice).
std::vector<int> forced_range_nodes() {
    std::vector<int> v;
    const char* e = std::getenv("HEC_TEST_RANGE_NODES");
    if (!e) return v;
    for (const char* c = e; *c;) {
        char* end;
        const long n = std::strtol(c, &end, 10);
        if (end == c) break;
        v.push_back(int(n));
        c = *end == ',' ? end + 1 : end;
    }
    return v;
}

}  // namespace hec

using namespace hec;

extern "C" {

int hec_device_numa_node(int device, int* node) {
    if (!node) return fail(HEC_ERR_INVALID_ARGUMENT, "null argument");
    *node = -1;
    int count = 0;
    if (hipGetDeviceCount(&count) != hipSuccess || count <= 0) {
        (void)hipGetLastError();
        return fail(HEC_ERR_NO_DEVICE, "no HIP device visible");
    }
    if (device < 0 || device >= count) return fail(HEC_ERR_INVALID_ARGUMENT, "device out of range");
    return device_numa_node(device, node);
}

int hec_bind_thread_to_device(int device, int* n_cpus) {
    if (n_cpus) *n_cpus = 0;
    int node = -1;
    int rc = hec_device_numa_node(device, &node);
    if (rc) return rc;
    if (node < 0) return HEC_OK;  // unknown node: nothing to bind to
    std::vector<int> cpus = parse_cpulist(read_line("/sys/devices/system/node/node" + std::to_string(node) +
                                                    "/cpulist"));
    cpu_set_t allowed, want;
    CPU_ZERO(&want);
    if (sched_getaffinity(0, sizeof(allowed), &allowed) != 0)
        return fail_errno(HEC_ERR_IO, "sched_getaffinity", errno);
    int n = 0;
    for (int c : cpus)
        if (c >= 0 && c < CPU_SETSIZE && CPU_ISSET(c, &allowed)) {
            CPU_SET(c, &want);
            ++n;
        }
    if (n == 0) return HEC_OK;  // none of the node's CPUs is ours (container cpuset): leave as is
    if (sched_setaffinity(0, sizeof(want), &want) != 0)
        return fail_errno(HEC_ERR_IO, "sched_setaffinity", errno);
    if (n_cpus) *n_cpus = n;
    return HEC_OK;
}

int hec_host_alloc(size_t bytes, void** out) {
    if (!out) return fail(HEC_ERR_INVALID_ARGUMENT, "null argument");
    *out = nullptr;
    if (bytes == 0) return fail(HEC_ERR_INVALID_ARGUMENT, "zero-byte allocation");
    return pinned_alloc(out, bytes);
}

int hec_host_alloc_multi(const int* devices, size_t n_devices, uint64_t stripe_stride, uint32_t n_stripes,
                         void** out) {
    if (!out) return fail(HEC_ERR_INVALID_ARGUMENT, "null argument");
    *out = nullptr;
    if (!devices || n_devices == 0 || n_devices > 256)
        return fail(HEC_ERR_INVALID_ARGUMENT, "device list must have 1..256 entries");
    uint64_t bytes;
    if (stripe_stride == 0 || n_stripes == 0 || __builtin_mul_overflow(stripe_stride, uint64_t(n_stripes), &bytes))
        return fail(HEC_ERR_INVALID_ARGUMENT, "empty or overflowing batch");
    int count = 0;
    HEC_TRY(hec_device_count(&count));
    for (size_t r = 0; r < n_devices; ++r)
        if (devices[r] < 0 || devices[r] >= count)
            return fail(HEC_ERR_INVALID_ARGUMENT, "device " + std::to_string(devices[r]) + " out of range");
    const uint64_t page = uint64_t(sysconf(_SC_PAGESIZE));
    const uint64_t len = (bytes + page - 1) / page * page;
    void* p = mmap(nullptr, len, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
    if (p == MAP_FAILED) return fail_errno(HEC_ERR_OUT_OF_MEMORY, "mmap", errno);
    // range r = stripes [S*r/R, S*(r+1)/R) -- the split hec_host_*_batch_multi
    // uses; a page that straddles two ranges goes with the earlier one
    const size_t R = std::min<size_t>(n_devices, n_stripes);
    const std::vector<int> forced = forced_range_nodes();
    const bool multi_node = online_nodes() >= 2;
    std::vector<std::pair<uint64_t, uint64_t>> spans(R);
    for (size_t r = 0; r < R; ++r) {
        const uint64_t s0 = uint64_t(n_stripes) * r / R, s1 = uint64_t(n_stripes) * (r + 1) / R;
        const uint64_t b0 = r == 0 ? 0 : std::min(len, (s0 * stripe_stride + page - 1) / page * page);
        const uint64_t b1 = r + 1 == R ? len : std::min(len, (s1 * stripe_stride + page - 1) / page * page);
        spans[r] = {b0, b1};
        int node = -1;
        if (r < forced.size()) node = forced[r];
        else (void)device_numa_node(devices[r], &node);
        if (!multi_node || node < 0 || node >= int(kMaxNodes) || b1 <= b0) continue;
        unsigned long mask[kMaskWords] = {0};
        mask[node / (8 * sizeof(unsigned long))] = 1ul << (node % (8 * sizeof(unsigned long)));
        // preferred, not bound: placement is speed only (a short node spills)
        (void)syscall(SYS_mbind, static_cast<uint8_t*>(p) + b0, b1 - b0, kMpolPreferred, mask, kMaxNodes, 0u);
    }
    // first touch under each range's policy, in parallel (the pool's threads
    // write; the policy belongs to the pages, not to the thread)
    constexpr uint64_t kTouch = 64ull << 20;
    const size_t pieces = size_t((len + kTouch - 1) / kTouch);
    parallel_for(pieces, len, [&](size_t i) {
        const uint64_t o = i * kTouch;
        std::memset(static_cast<uint8_t*>(p) + o, 0, size_t(std::min(kTouch, len - o)));
    });
    const hipError_t e = hipHostRegister(p, len, hipHostRegisterMapped | hipHostRegisterPortable);
    if (e != hipSuccess) {
        munmap(p, len);
        return hip_fail(e, "hipHostRegister");
    }
    {
        std::lock_guard<std::mutex> lk(placed_mu());
        placed_allocs()[p] = size_t(len);
    }
    *out = p;
    return HEC_OK;
}

int hec_host_free(void* p) {
    if (!p) return HEC_OK;
    size_t len = 0;
    {
        std::lock_guard<std::mutex> lk(placed_mu());
        auto it = placed_allocs().find(p);
        if (it != placed_allocs().end()) {
            len = it->second;
            placed_allocs().erase(it);
        }
    }
    if (len) {  // a hec_host_alloc_multi batch
        const hipError_t e = hipHostUnregister(p);
        munmap(p, len);
        if (e != hipSuccess) return hip_fail(e, "hipHostUnregister");
        return HEC_OK;
    }
    HEC_HIP(hipHostFree(p));
    return HEC_OK;
}

int hec_host_numa_node(const void* p, int* node) {
    if (!p || !node) return fail(HEC_ERR_INVALID_ARGUMENT, "null argument");
    *node = -1;
    void* page = reinterpret_cast<void*>(reinterpret_cast<uintptr_t>(p) & ~uintptr_t(sysconf(_SC_PAGESIZE) - 1));
    int status = -1;
    // move_pages with nodes == NULL only reports where each page lives
    if (syscall(SYS_move_pages, 0, 1ul, &page, nullptr, &status, 0) != 0)
        return fail_errno(HEC_ERR_IO, "move_pages", errno);
    if (status < 0) return fail_errno(HEC_ERR_IO, "page not resident", -status);
    *node = status;
    return HEC_OK;
}

}  // extern "C"
