// mpx_counters.cpp — libmpxprof.so: hardware counters of this process's own
// GPU work, read from inside the process with rocprofiler-sdk's DEVICE
// counting service (include/mpxprof.h).
//
// Why in-process (VERDICT r03 "Next round" 1): rocprofv3 --pmc is the
// dispatch counting service; it serialises dispatches, so it cannot run the
// two co-dependent halves of a pair in one process, and bench.py's own
// multi-GPU line could not carry counters.  The device counting service
// reads agent-wide counters between two samples and leaves dispatch alone.
//
// Life cycle: mpxprof_register() (before HIP starts) hands tool_configure to
// rocprofiler_force_configure; when the HSA runtime initialises, tool_init
// creates one context per GPU agent with the device counting service
// configured on it (contexts and services can only be set up there).
// mpxprof_begin() picks the agent by PCI bus id, builds (and caches) the
// counter config, starts the context — its set-config callback installs the
// config — and takes a baseline sample; mpxprof_end() samples and stops.
//
// Used by bench.py only, around untimed re-runs of the measured work; never
// inside a timed region.  Not part of libmpx (the drop-in path).
#include "../../include/mpxprof.h"

#include <rocprofiler-sdk/registration.h>
#include <rocprofiler-sdk/rocprofiler.h>

#include <execinfo.h>
#include <signal.h>
#include <unistd.h>

#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>
#include <string>
#include <vector>

namespace {

struct Agent {
    rocprofiler_agent_id_t id{};
    uint32_t domain = 0, location = 0;      // PCI domain, BDF = bus<<8 | dev<<3 | fn
    rocprofiler_context_id_t ctx{};
    rocprofiler_counter_config_id_t pending{};   // installed at context start
    std::map<std::string, rocprofiler_counter_id_t> supported;   // name -> id (filled on first use)
    std::map<std::string, rocprofiler_counter_config_id_t> configs;
};

std::mutex g_mu;
std::vector<Agent>* g_agents = new std::vector<Agent>;   // never destroyed (no exit-order hazards)
bool g_ready = false;
std::string g_err;
// the pass in progress
Agent* g_active = nullptr;
std::vector<rocprofiler_counter_id_t> g_want;
std::vector<double> g_base;

int fail(const char* fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    g_err = buf;
    return -1;
}

#define RP(expr, what)                                                                  \
    do {                                                                                \
        const rocprofiler_status_t s_ = (expr);                                         \
        if (s_ != ROCPROFILER_STATUS_SUCCESS)                                           \
            return fail("%s: %s", what, rocprofiler_get_status_string(s_));             \
    } while (0)

void set_config_cb(rocprofiler_context_id_t ctx, rocprofiler_agent_id_t, rocprofiler_device_counting_agent_cb_t set,
                   void* user) {
    Agent* a = static_cast<Agent*>(user);
    if (a && a->pending.handle) set(ctx, a->pending);
}

rocprofiler_status_t collect_agents(rocprofiler_agent_version_t ver, const void** arr, size_t n, void* user) {
    if (ver != ROCPROFILER_AGENT_INFO_VERSION_0) return ROCPROFILER_STATUS_ERROR;
    auto* out = static_cast<std::vector<Agent>*>(user);
    for (size_t i = 0; i < n; ++i) {
        const auto* ag = static_cast<const rocprofiler_agent_v0_t*>(arr[i]);
        if (ag->type != ROCPROFILER_AGENT_TYPE_GPU) continue;
        Agent a;
        a.id = ag->id;
        a.domain = ag->domain;
        a.location = ag->location_id;
        out->push_back(a);
    }
    return ROCPROFILER_STATUS_SUCCESS;
}

int tool_init(rocprofiler_client_finalize_t, void*) {
    std::lock_guard<std::mutex> lk(g_mu);
    std::vector<Agent>& agents = *g_agents;
    if (rocprofiler_query_available_agents(ROCPROFILER_AGENT_INFO_VERSION_0, collect_agents, sizeof(rocprofiler_agent_t),
                                           &agents) != ROCPROFILER_STATUS_SUCCESS || agents.empty()) {
        fail("no GPU agent");
        return 0;   // the process runs on; mpxprof_ready() stays 0
    }
    // the vector is not resized after this point: the callbacks keep &agents[i]
    for (Agent& a : agents) {
        if (rocprofiler_create_context(&a.ctx) != ROCPROFILER_STATUS_SUCCESS) {
            fail("rocprofiler_create_context failed");
            return 0;
        }
        const rocprofiler_status_t s =
            rocprofiler_configure_device_counting_service(a.ctx, rocprofiler_buffer_id_t{0}, a.id, set_config_cb, &a);
        if (s != ROCPROFILER_STATUS_SUCCESS) {
            fail("rocprofiler_configure_device_counting_service: %s", rocprofiler_get_status_string(s));
            return 0;
        }
    }
    g_ready = true;
    return 0;
}

void tool_fini(void*) {
    std::lock_guard<std::mutex> lk(g_mu);
    if (g_active) (void)rocprofiler_stop_context(g_active->ctx);
    g_active = nullptr;
    g_ready = false;
}

rocprofiler_tool_configure_result_t* tool_configure(uint32_t, const char*, uint32_t, rocprofiler_client_id_t* id) {
    id->name = "mpxprof";
    static rocprofiler_tool_configure_result_t cfg{sizeof(rocprofiler_tool_configure_result_t), &tool_init,
                                                   &tool_fini, nullptr};
    return &cfg;
}

rocprofiler_status_t collect_counters(rocprofiler_agent_id_t, rocprofiler_counter_id_t* c, size_t n, void* user) {
    auto* m = static_cast<std::map<std::string, rocprofiler_counter_id_t>*>(user);
    for (size_t i = 0; i < n; ++i) {
        rocprofiler_counter_info_v0_t info{};
        if (rocprofiler_query_counter_info(c[i], ROCPROFILER_COUNTER_INFO_VERSION_0, &info) == ROCPROFILER_STATUS_SUCCESS &&
            info.name)
            (*m)[info.name] = c[i];
    }
    return ROCPROFILER_STATUS_SUCCESS;
}

Agent* find_agent(const char* bus_id) {
    unsigned dom = 0, bus = 0, dev = 0, fn = 0;
    if (!bus_id || sscanf(bus_id, "%x:%x:%x.%x", &dom, &bus, &dev, &fn) != 4) {
        fail("bad PCI bus id '%s'", bus_id ? bus_id : "(null)");
        return nullptr;
    }
    const uint32_t loc = (bus << 8) | (dev << 3) | fn;
    for (Agent& a : *g_agents)
        if (a.domain == dom && a.location == loc) return &a;
    fail("no GPU agent at %s", bus_id);
    return nullptr;
}

std::vector<std::string> split(const char* s) {
    std::vector<std::string> out;
    std::string cur;
    for (const char* p = s; p && *p; ++p) {
        if (*p == ',') {
            if (!cur.empty()) out.push_back(cur);
            cur.clear();
        } else if (*p != ' ') {
            cur += *p;
        }
    }
    if (!cur.empty()) out.push_back(cur);
    return out;
}

// one sample of the active pass: per wanted counter, the sum over its records
int sample(std::vector<double>& out) {
    std::vector<rocprofiler_counter_record_t> rec(1 << 14);
    size_t n = rec.size();
    RP(rocprofiler_sample_device_counting_service(g_active->ctx, rocprofiler_user_data_t{}, ROCPROFILER_COUNTER_FLAG_NONE,
                                                  rec.data(), &n),
       "rocprofiler_sample_device_counting_service");
    out.assign(g_want.size(), 0.0);
    for (size_t i = 0; i < n; ++i) {
        rocprofiler_counter_id_t cid{};
        if (rocprofiler_query_record_counter_id(rec[i].id, &cid) != ROCPROFILER_STATUS_SUCCESS) continue;
        for (size_t k = 0; k < g_want.size(); ++k)
            if (g_want[k].handle == cid.handle) out[k] += rec[i].counter_value;
    }
    return 0;
}

}  // namespace

extern "C" {

// Diagnostics: a process that registers the tool and later dies of SIGSEGV
// prints the faulting thread's native stack to stderr first (then the default
// action runs), so an exit-time crash names the library it happened in.
void segv_dump(int sig) {
    void* frames[64];
    const int n = backtrace(frames, 64);
    const char msg[] = "[mpxprof] fatal signal; native stack:\n";
    (void)!write(2, msg, sizeof msg - 1);
    backtrace_symbols_fd(frames, n, 2);
    signal(sig, SIG_DFL);
    raise(sig);
}

int mpxprof_register(void) {
    if (getenv("MPXPROF_SEGV_DUMP")) {
        signal(SIGSEGV, segv_dump);
        signal(SIGABRT, segv_dump);
    }
    const rocprofiler_status_t s = rocprofiler_force_configure(&tool_configure);
    if (s != ROCPROFILER_STATUS_SUCCESS) return fail("rocprofiler_force_configure: %s", rocprofiler_get_status_string(s));
    return 0;
}

int mpxprof_ready(void) {
    std::lock_guard<std::mutex> lk(g_mu);
    return g_ready ? 1 : 0;
}

const char* mpxprof_error(void) { return g_err.c_str(); }

int mpxprof_begin(const char* bus_id, const char* counters) {
    std::lock_guard<std::mutex> lk(g_mu);
    if (!g_ready) return g_err.empty() ? fail("the tool was not initialised (register before HIP starts)") : -1;
    if (g_active) return fail("a pass is already running");
    Agent* a = find_agent(bus_id);
    if (!a) return -1;
    if (a->supported.empty()) {
        RP(rocprofiler_iterate_agent_supported_counters(a->id, collect_counters, &a->supported),
           "rocprofiler_iterate_agent_supported_counters");
    }
    const std::vector<std::string> names = split(counters);
    if (names.empty()) return fail("no counters named");
    std::vector<rocprofiler_counter_id_t> ids;
    for (const std::string& nm : names) {
        auto it = a->supported.find(nm);
        if (it == a->supported.end()) return fail("counter %s is not supported on this agent", nm.c_str());
        ids.push_back(it->second);
    }
    auto ct = a->configs.find(counters);
    if (ct == a->configs.end()) {
        rocprofiler_counter_config_id_t cfg{};
        RP(rocprofiler_create_counter_config(a->id, ids.data(), ids.size(), &cfg), "rocprofiler_create_counter_config");
        ct = a->configs.emplace(counters, cfg).first;
    }
    a->pending = ct->second;
    RP(rocprofiler_start_context(a->ctx), "rocprofiler_start_context");
    g_active = a;
    g_want = ids;
    if (sample(g_base) != 0) {
        (void)rocprofiler_stop_context(a->ctx);
        g_active = nullptr;
        return -1;
    }
    return 0;
}

int mpxprof_end(double* values, int n, int* reads_reset) {
    std::lock_guard<std::mutex> lk(g_mu);
    if (!g_active) return fail("no pass is running");
    std::vector<double> s1, s2;
    int rc = sample(s1);
    if (rc == 0) rc = sample(s2);   // right after s1: tells cumulative from reset-on-read samples
    (void)rocprofiler_stop_context(g_active->ctx);
    g_active = nullptr;
    if (rc != 0) return -1;
    // cumulative: s2 repeats s1 (nothing ran between them); reset-on-read:
    // s2 holds only what ran between the two reads, ~0
    double a1 = 0, a2 = 0;
    for (size_t k = 0; k < s1.size(); ++k) {
        a1 += std::fabs(s1[k]);
        a2 += std::fabs(s2[k]);
    }
    const bool reset = a1 > 0 && a2 < 0.5 * a1;
    if (reads_reset) *reads_reset = reset ? 1 : 0;
    for (int k = 0; k < n && k < (int)s1.size(); ++k) values[k] = reset ? s1[k] : s1[k] - g_base[k];
    return 0;
}

}  // extern "C"
