// NUMA placement of the host side of each GPU (one host thread
// + stream + NUMA-local pinned buffers per GPU). helyim itself is CPU-only and
// NUMA-unaware; the GPU path adds PCIe and host-DRAM traffic per GPU, so every
// pinned buffer this library allocates lives on the NUMA node of the GPU that
// reads it over PCIe, and a caller (one process or thread per GPU) can bind its
// CPUs to that node too.
//
// Node of a GPU: sysfs numa_node of its PCI function (hipDeviceGetPCIBusId).
// Placement: the allocating thread's memory policy is set to MPOL_BIND on that
// node around hipHostMalloc(hipHostMallocNumaUser), which makes the runtime
// follow the thread's policy when it backs the pinned range, then restored.
// Raw syscalls, so libhec needs no libnuma.
#include <sched.h>
#include <sys/syscall.h>
#include <unistd.h>

#include <cctype>
#include <cstdlib>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <string>
#include <vector>

#include "hec_internal.hpp"

namespace hec {
namespace {

constexpr int kMpolDefault = 0;
constexpr int kMpolBind = 2;
constexpr unsigned kMaxNodes = 1024;

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

// Test hook: HEC_TEST_NUMA_BIND_FAIL=1 makes every NUMA-bound allocation
// attempt fail as if the node were full, so the fallback below runs on any
// machine (tests/test_gpu_numa.py).
static bool bind_failure_forced() {
    static const bool forced = [] {
        const char* v = std::getenv("HEC_TEST_NUMA_BIND_FAIL");
        return v && v[0] == '1';
    }();
    return forced;
}

// Pinned host memory on the current device's NUMA node (plain hipHostMalloc
// when the node is unknown or the machine has one node). Placement is a speed
// preference, never a requirement: when the node cannot back the range
// (MPOL_BIND and its free memory is short), the allocation is retried under
// the default policy (any node) instead of failing.
int pinned_alloc(void** p, size_t bytes) {
    *p = nullptr;
    int dev, node = -1, rc;
    if ((rc = current_device(&dev))) return rc;
    if ((rc = device_numa_node(dev, &node))) return rc;
    const bool forced = bind_failure_forced();
    if (!forced && (node < 0 || node >= int(kMaxNodes) || online_nodes() < 2)) {
        HEC_HIP(hipHostMalloc(p, bytes, hipHostMallocDefault));
        return HEC_OK;
    }
    if (forced) {
        HEC_HIP(hipHostMalloc(p, bytes, hipHostMallocDefault));  // the fallback's allocation
        return HEC_OK;
    }
    unsigned long old_mask[kMaxNodes / (8 * sizeof(unsigned long))] = {0};
    int old_mode = kMpolDefault;
    const bool saved = syscall(SYS_get_mempolicy, &old_mode, old_mask, kMaxNodes, nullptr, 0) == 0;
    unsigned long mask[kMaxNodes / (8 * sizeof(unsigned long))] = {0};
    mask[node / (8 * sizeof(unsigned long))] = 1ul << (node % (8 * sizeof(unsigned long)));
    const bool bound = syscall(SYS_set_mempolicy, kMpolBind, mask, kMaxNodes) == 0;
    hipError_t e = hipHostMalloc(p, bytes, bound ? hipHostMallocNumaUser : hipHostMallocDefault);
    if (bound) {
        if (saved) (void)syscall(SYS_set_mempolicy, old_mode, old_mode == kMpolDefault ? nullptr : old_mask,
                                 kMaxNodes);
        else (void)syscall(SYS_set_mempolicy, kMpolDefault, nullptr, 0);
    }
    if (e == hipSuccess) return HEC_OK;
    (void)hipGetLastError();
    *p = nullptr;
    e = hipHostMalloc(p, bytes, hipHostMallocDefault);  // any node: placement is speed only
    if (e != hipSuccess) return hip_fail(e, "hipHostMalloc (pinned, after the NUMA-local attempt failed)");
    return HEC_OK;
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
        return fail(HEC_ERR_IO, std::string("sched_getaffinity: ") + strerror(errno));
    int n = 0;
    for (int c : cpus)
        if (c >= 0 && c < CPU_SETSIZE && CPU_ISSET(c, &allowed)) {
            CPU_SET(c, &want);
            ++n;
        }
    if (n == 0) return HEC_OK;  // none of the node's CPUs is ours (container cpuset): leave as is
    if (sched_setaffinity(0, sizeof(want), &want) != 0)
        return fail(HEC_ERR_IO, std::string("sched_setaffinity: ") + strerror(errno));
    if (n_cpus) *n_cpus = n;
    return HEC_OK;
}

int hec_host_alloc(size_t bytes, void** out) {
    if (!out) return fail(HEC_ERR_INVALID_ARGUMENT, "null argument");
    *out = nullptr;
    if (bytes == 0) return fail(HEC_ERR_INVALID_ARGUMENT, "zero-byte allocation");
    return pinned_alloc(out, bytes);
}

int hec_host_free(void* p) {
    if (!p) return HEC_OK;
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
        return fail(HEC_ERR_IO, std::string("move_pages: ") + strerror(errno));
    if (status < 0) return fail(HEC_ERR_IO, std::string("page not resident: ") + strerror(-status));
    *node = status;
    return HEC_OK;
}

}  // extern "C"
