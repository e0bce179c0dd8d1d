// Development probe (not product code): how the GPU box's two NUMA nodes shape
// the host side of the ingest pipeline.
//   1. the device's node (sysfs, from its PCI bus id) and where hipHostMalloc
//      places pinned pages (move_pages query);
//   2. H2D rate from pinned memory bound to each node (mmap + mbind + hipHostRegister);
//   3. memcpy rate with 8 threads pinned to node t, source on node s, target on node d.
//
//   hipcc -O2 -std=c++17 tools/numa_probe.cpp -o build/numa_probe && build/numa_probe
#include <hip/hip_runtime.h>
#include <sched.h>
#include <sys/mman.h>
#include <sys/syscall.h>
#include <unistd.h>

#include <chrono>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <string>
#include <thread>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); exit(1); } } while (0)

static const size_t MB = 1 << 20;

static std::vector<int> parse_list(const std::string &s) {
    std::vector<int> v;
    size_t i = 0;
    while (i < s.size()) {
        size_t j = s.find(',', i);
        if (j == std::string::npos) j = s.size();
        std::string r = s.substr(i, j - i);
        size_t d = r.find('-');
        if (!r.empty() && r[0] >= '0' && r[0] <= '9') {
            int a = std::stoi(r), b = d == std::string::npos ? a : std::stoi(r.substr(d + 1));
            for (int k = a; k <= b; k++) v.push_back(k);
        }
        i = j + 1;
    }
    return v;
}

static std::vector<int> node_cpus(int node) {
    std::ifstream f("/sys/devices/system/node/node" + std::to_string(node) + "/cpulist");
    std::string s;
    std::getline(f, s);
    return parse_list(s);
}

static void bind_thread(int node) {
    cpu_set_t cs;
    CPU_ZERO(&cs);
    for (int c : node_cpus(node)) CPU_SET(c, &cs);
    sched_setaffinity(0, sizeof(cs), &cs);
}

static void *alloc_on(int node, size_t n) {
    void *p = mmap(nullptr, n, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
    unsigned long mask = 1ul << node;
    if (syscall(SYS_mbind, p, n, 2 /*MPOL_BIND*/, &mask, 64, 0) != 0) perror("mbind");
    memset(p, 1, n);
    return p;
}

static std::vector<int> page_nodes(void *p, size_t n, int samples) {
    std::vector<void *> pages(samples);
    std::vector<int> st(samples, -99);
    for (int i = 0; i < samples; i++) pages[i] = (char *)p + (n / samples) * i;
    syscall(SYS_move_pages, 0, samples, pages.data(), nullptr, st.data(), 0);
    return st;
}

static double now() {
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

// busy fraction of each node's CPUs over 0.5 s (/proc/stat): other tenants' load
static void node_load(double out[2]) {
    auto snap = [](std::vector<std::pair<long long, long long>> &v) {
        std::ifstream f("/proc/stat");
        std::string line;
        v.assign(512, {0, 0});
        while (std::getline(f, line)) {
            if (line.compare(0, 3, "cpu") || line[3] < '0' || line[3] > '9') continue;
            int c = std::stoi(line.substr(3));
            long long x[10] = {0};
            sscanf(line.c_str() + line.find(' '), "%lld %lld %lld %lld %lld %lld %lld %lld", x, x + 1, x + 2, x + 3,
                   x + 4, x + 5, x + 6, x + 7);
            long long tot = 0;
            for (int k = 0; k < 8; k++) tot += x[k];
            if (c < 512) v[c] = {tot, x[3] + x[4]};
        }
    };
    std::vector<std::pair<long long, long long>> a, b;
    snap(a);
    usleep(500000);
    snap(b);
    for (int n = 0; n < 2; n++) {
        long long tot = 0, idle = 0;
        for (int c : node_cpus(n)) tot += b[c].first - a[c].first, idle += b[c].second - a[c].second;
        out[n] = tot ? 1.0 - (double)idle / (double)tot : 0;
    }
}

int main() {
    char bus[64];
    CK(hipSetDevice(0));
    CK(hipDeviceGetPCIBusId(bus, sizeof bus, 0));
    std::string b(bus);
    for (auto &c : b) c = (char)tolower(c);
    std::ifstream nf("/sys/bus/pci/devices/" + b + "/numa_node");
    int gnode = -1;
    nf >> gnode;
    double ld[2];
    node_load(ld);
    printf("{\"device_bus\": \"%s\", \"device_node\": %d, \"node_busy\": [%.3f, %.3f]", b.c_str(), gnode, ld[0], ld[1]);
    const size_t N = 256 * MB;
    void *pin;
    CK(hipHostMalloc(&pin, N, 0));
    memset(pin, 2, N);
    auto st = page_nodes(pin, N, 64);
    int c0 = 0, c1 = 0;
    for (int s : st) c0 += s == 0, c1 += s == 1;
    printf(", \"hipHostMalloc_pages_node0\": %d, \"node1\": %d", c0, c1);
    void *dev;
    CK(hipMalloc(&dev, N));
    hipStream_t s;
    CK(hipStreamCreate(&s));
    auto h2d = [&](void *src) {
        CK(hipMemcpyAsync(dev, src, N, hipMemcpyHostToDevice, s));
        CK(hipStreamSynchronize(s));
        double best = 0;
        for (int r = 0; r < 8; r++) {
            double t = now();
            CK(hipMemcpyAsync(dev, src, N, hipMemcpyHostToDevice, s));
            CK(hipStreamSynchronize(s));
            best = std::max(best, N / (now() - t) / 1e9);
        }
        return best;
    };
    printf(", \"h2d_hipHostMalloc_GBs\": %.2f", h2d(pin));
    for (int node = 0; node < 2; node++) {
        void *p = alloc_on(node, N);
        CK(hipHostRegister(p, N, 0));
        printf(", \"h2d_node%d_GBs\": %.2f", node, h2d(p));
        CK(hipHostUnregister(p));
        munmap(p, N);
    }
    // memcpy: 8 threads on node t, 1 GiB from node s to node d (best of 3)
    const size_t M = 1024 * MB;
    void *src[2] = {alloc_on(0, M), alloc_on(1, M)}, *dst[2] = {alloc_on(0, M), alloc_on(1, M)};
    for (int t = 0; t < 2; t++)
        for (int sn = 0; sn < 2; sn++)
            for (int dn = 0; dn < 2; dn++) {
                double best = 0;
                for (int r = 0; r < 3; r++) {
                    std::vector<std::thread> th;
                    double t0 = now();
                    for (int k = 0; k < 8; k++)
                        th.emplace_back([&, k] {
                            bind_thread(t);
                            memcpy((char *)dst[dn] + k * (M / 8), (char *)src[sn] + k * (M / 8), M / 8);
                        });
                    for (auto &x : th) x.join();
                    best = std::max(best, M / (now() - t0) / 1e9);
                }
                printf(", \"copy_t%d_s%d_d%d_GBs\": %.2f", t, sn, dn, best);
            }
    // the pipeline's shape: H2D from the pinned buffer while 8 threads copy into another pinned buffer
    for (int t = 0; t < 2; t++) {
        void *pin2;
        CK(hipHostMalloc(&pin2, M, 0));
        memset(pin2, 3, M);
        double t0 = now();
        for (int r = 0; r < 4; r++) CK(hipMemcpyAsync(dev, pin, N, hipMemcpyHostToDevice, s));
        std::vector<std::thread> th;
        for (int k = 0; k < 8; k++)
            th.emplace_back([&, k] {
                bind_thread(t);
                memcpy((char *)pin2 + k * (M / 8), (char *)src[gnode == 1 ? 1 : 0] + k * (M / 8), M / 8);
            });
        for (auto &x : th) x.join();
        double tc = now() - t0;
        CK(hipStreamSynchronize(s));
        double td = now() - t0;
        printf(", \"overlap_t%d\": {\"copy_GBs\": %.2f, \"h2d_GBs\": %.2f}", t, M / tc / 1e9, 4.0 * N / td / 1e9);
        CK(hipHostFree(pin2));
    }
    printf("}\n");
    return 0;
}
