// Library-level C ABI: error text, version, and the in-library kernel timer.
#include <cstdarg>
#include <cstdio>
#include <map>
#include <mutex>
#include <string>
#include <vector>

#include "common.h"

namespace spn {

static thread_local char g_err[1024] = "";

void set_error(const char* fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof(g_err), fmt, ap);
    va_end(ap);
}

// ---- profiler: per kernel class, HIP event pairs recorded on the launch stream ------------
struct Rec {
    hipEvent_t a, b;
    double flop, bytes;
};
struct ClassStats {
    std::vector<Rec> pending;
    int64_t launches = 0;
    double ms = 0, flop = 0, bytes = 0;
};
static std::mutex g_mu;
static bool g_on = false;
static std::map<std::string, ClassStats> g_stats;
static std::vector<hipEvent_t> g_pool;

static hipEvent_t take_event() {
    if (!g_pool.empty()) {
        hipEvent_t e = g_pool.back();
        g_pool.pop_back();
        return e;
    }
    hipEvent_t e = nullptr;
    if (hipEventCreate(&e) != hipSuccess) return nullptr;
    return e;
}

int g_prof_shapes = 0;

int num_cus() {
    static int cached[64] = {0};
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 256;
    if (cached[dev] <= 0) {
        int n = 0;
        if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) n = 256;
        cached[dev] = n;
    }
    return cached[dev];
}

ProfScope::ProfScope(const char* cls, hipStream_t s, double flop, double bytes) : rec_(nullptr), s_(s) {
    if (!g_on) return;
    std::lock_guard<std::mutex> lk(g_mu);
    Rec* r = new Rec{take_event(), take_event(), flop, bytes};
    if (!r->a || !r->b || hipEventRecord(r->a, s) != hipSuccess) {
        delete r;
        return;
    }
    std::string key(cls);
    if (g_prof_shapes) key += "#" + std::to_string((long long)(flop / 1e6 + 0.5)) + "MF";
    auto& st = g_stats[key];
    st.pending.push_back(*r);
    delete r;
    rec_ = (void*)&st;
}

ProfScope::~ProfScope() {
    if (!rec_) return;
    std::lock_guard<std::mutex> lk(g_mu);
    auto* st = (ClassStats*)rec_;
    (void)hipEventRecord(st->pending.back().b, s_);
}

static void drain(ClassStats& st) {
    for (auto& r : st.pending) {
        float ms = 0.f;
        (void)hipEventSynchronize(r.b);
        if (hipEventElapsedTime(&ms, r.a, r.b) == hipSuccess) {
            st.ms += ms;
            st.flop += r.flop;
            st.bytes += r.bytes;
            st.launches += 1;
        }
        g_pool.push_back(r.a);
        g_pool.push_back(r.b);
    }
    st.pending.clear();
}

}  // namespace spn

using namespace spn;

extern "C" const char* spnerf_last_error(void) { return g_err; }

extern "C" int32_t spnerf_abi_version(void) { return 2; }

extern "C" int32_t spnerf_prof_enable(int32_t on) {
    std::lock_guard<std::mutex> lk(g_mu);
    g_on = on != 0;
    return SPNERF_OK;
}

extern "C" int32_t spnerf_prof_reset(void) {
    std::lock_guard<std::mutex> lk(g_mu);
    for (auto& kv : g_stats) drain(kv.second);
    g_stats.clear();
    return SPNERF_OK;
}

extern "C" int32_t spnerf_prof_classes(char* buf, int32_t cap) {
    SPN_ARG(buf != nullptr && cap > 0, "prof_classes: NULL buffer");
    std::lock_guard<std::mutex> lk(g_mu);
    std::string names;
    for (auto& kv : g_stats) names += (names.empty() ? "" : ",") + kv.first;
    SPN_ARG((int64_t)names.size() < cap, "prof_classes: buffer of %d bytes too small (%zu)", cap, names.size() + 1);
    snprintf(buf, cap, "%s", names.c_str());
    return SPNERF_OK;
}

extern "C" int32_t spnerf_prof_read(const char* cls, int64_t* launches, double* total_ms, double* total_flop,
                                    double* total_bytes) {
    SPN_ARG(cls != nullptr, "prof_read: NULL class");
    std::lock_guard<std::mutex> lk(g_mu);
    auto it = g_stats.find(cls);
    if (it == g_stats.end()) {
        if (launches) *launches = 0;
        if (total_ms) *total_ms = 0;
        if (total_flop) *total_flop = 0;
        if (total_bytes) *total_bytes = 0;
        return SPNERF_OK;
    }
    drain(it->second);
    if (launches) *launches = it->second.launches;
    if (total_ms) *total_ms = it->second.ms;
    if (total_flop) *total_flop = it->second.flop;
    if (total_bytes) *total_bytes = it->second.bytes;
    return SPNERF_OK;
}
