// opts.cpp -- engine options of a context (dev.hpp: EngineOpts).  A context copies the
// CPK_<NAME> environment variables once at creation; cpk_ctx_set_option changes its copy.
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>

#include "dev.hpp"

namespace cpk {

namespace {

bool parse_bool(const std::string &name, const std::string &v) {
    if (v.empty() || v == "1" || v == "true" || v == "on" || v == "yes") return true;
    if (v == "0" || v == "false" || v == "off" || v == "no") return false;
    char *end = nullptr;
    const long x = strtol(v.c_str(), &end, 10);
    if (end && *end == '\0') return x != 0;
    throw Error(CPK_ERR_ARGS, "engine option " + name + ": not a boolean: '" + v + "'");
}

SweepConfig parse_sweep(const std::string &v) {
    SweepConfig cfg;
    int a[7] = {0, 0, 0, 0, 0, 0, 0};
    const int got = sscanf(v.c_str(), "%d,%d,%d,%d,%d,%d,%d", &a[0], &a[1], &a[2], &a[3], &a[4], &a[5], &a[6]);
    if (got == 3) a[3] = a[0], a[4] = a[1], a[5] = a[2];
    auto ok = [](int r, int c, int t) {
        return r > 0 && r <= 16384 && c > 0 && c <= 16384 &&
               (t == 32 || t == 64 || t == 128 || t == 256 || t == 512 || t == 1024) &&
               sweep_lds_bytes(r, c) <= 160 * 1024;
    };
    if (!((got == 3 || got == 6 || got == 7) && ok(a[0], a[1], a[2]) && ok(a[3], a[4], a[5])))
        throw Error(CPK_ERR_ARGS, "engine option sweep: expected rows,cap,threads[,rows,cap,threads[,sub0]] "
                                  "(threads 32..1024, LDS image <= 160 KB), got '" + v + "'");
    for (int i = 0; i < 2; i++) cfg.rows[i] = a[3 * i], cfg.cap[i] = a[3 * i + 1], cfg.threads[i] = a[3 * i + 2];
    cfg.sub0 = got == 7 ? a[6] : 0;
    return cfg;
}

std::string sweep_str(const SweepConfig &c) {
    char b[128];
    snprintf(b, sizeof b, "%d,%d,%d,%d,%d,%d,%d", c.rows[0], c.cap[0], c.threads[0], c.rows[1], c.cap[1], c.threads[1],
             c.sub0);
    return b;
}

// the boolean options: name -> member
struct BoolOpt {
    const char *name;
    bool EngineOpts::*m;
};
const BoolOpt kBool[] = {
    {"host_factor", &EngineOpts::host_factor},
    {"no_pipe", &EngineOpts::no_pipe},
    {"no_upper", &EngineOpts::no_upper},
    {"no_col16", &EngineOpts::no_col16},
    {"no_dataflow", &EngineOpts::no_dataflow},
    {"all_dataflow", &EngineOpts::all_dataflow},
    {"no_colsweep", &EngineOpts::no_colsweep},
    {"all_colsweep", &EngineOpts::all_colsweep},
    {"no_sched_resid", &EngineOpts::no_sched_resid},
    {"no_fused_resid", &EngineOpts::no_fused_resid},
    {"tsolve_global", &EngineOpts::tsolve_global},
    {"tsolve_sweep", &EngineOpts::tsolve_sweep},
    {"no_piggy", &EngineOpts::no_piggy},
    {"no_halo_merge", &EngineOpts::no_halo_merge},
    {"no_graph", &EngineOpts::no_graph},
    {"no_fuse_last", &EngineOpts::no_fuse_last},
    {"no_tkr", &EngineOpts::no_tkr},
    {"no_minres_fuse", &EngineOpts::no_minres_fuse},
    {"dist_graph", &EngineOpts::dist_graph},
    {"dist1", &EngineOpts::dist1},
    {"exact_dots", &EngineOpts::exact_dots},
    {"no_chain", &EngineOpts::no_chain},
    {"no_bcast_analysis", &EngineOpts::no_bcast_analysis},
    {"profile_fwd_sched", &EngineOpts::profile_fwd_sched},
    {"profile_passes", &EngineOpts::profile_passes},
};

}  // namespace

SweepConfig dist_sweep_default() {
    SweepConfig c;
    c.rows[0] = 192, c.cap[0] = 576, c.threads[0] = 64;
    c.rows[1] = 1024, c.cap[1] = 4096, c.threads[1] = 512;
    c.sub0 = 0;
    return c;
}

SweepConfig effective_sweep(const EngineOpts &o, bool dist) { return (dist && !o.sweep_set) ? dist_sweep_default() : o.sweep; }

void set_engine_option(EngineOpts &o, const std::string &name, const std::string &value) {
    for (const BoolOpt &b : kBool)
        if (name == b.name) {
            o.*b.m = parse_bool(name, value);
            return;
        }
    if (name == "sweep") {
        o.sweep = parse_sweep(value);
        o.sweep_set = true;
    } else if (name == "sweep_set") {  // engine_opts_string's round trip: "0" restores the per-path default
        o.sweep_set = parse_bool(name, value);
    } else if (name == "split_tol") {
        char *end = nullptr;
        const double v = strtod(value.c_str(), &end);
        if (end == value.c_str() || *end != '\0' || !std::isfinite(v) || !(v > 0 && v < 1))
            throw Error(CPK_ERR_ARGS, "engine option split_tol must be a number in (0, 1), got '" + value + "'");
        o.split_tol = v;
    } else if (name == "batch" || name == "r0_xcd_chunk") {
        char *end = nullptr;
        const long v = strtol(value.c_str(), &end, 10);
        if (end == value.c_str() || *end != '\0' || v < 0 || v > 4096)
            throw Error(CPK_ERR_ARGS, "engine option " + name + " must be an integer in [0, 4096], got '" + value + "'");
        (name == "batch" ? o.batch : o.r0_xcd_chunk) = (int)v;
    } else if (name == "fail_inject") {  // test hook (dev.hpp): "R:setup", "R:batch:K" or "R:chain:K"
        int r = -1, k = 0;
        char site[16] = {0};
        const bool ok = value.empty() ||
                        (sscanf(value.c_str(), "%d:%15[a-z]:%d", &r, site, &k) >= 2 && r >= 0 &&
                         (std::string(site) == "setup" || std::string(site) == "batch" || std::string(site) == "chain"));
        if (!ok)
            throw Error(CPK_ERR_ARGS, "engine option fail_inject: expected R:setup, R:batch:K or R:chain:K, got '" + value + "'");
        o.fail_inject = value;
    } else if (name == "chain_wide") {
        char *end = nullptr;
        const long v = strtol(value.c_str(), &end, 10);
        if (end == value.c_str() || *end != '\0' || v < 1 || v > (1L << 24))
            throw Error(CPK_ERR_ARGS, "engine option chain_wide must be an integer in [1, 2^24], got '" + value + "'");
        o.chain_wide = (int)v;
    } else {
        throw Error(CPK_ERR_ARGS, "unknown engine option '" + name + "'");
    }
}

std::string get_engine_option(const EngineOpts &o, const std::string &name, bool dist) {
    for (const BoolOpt &b : kBool)
        if (name == b.name) return o.*b.m ? "1" : "0";
    if (name == "sweep") return sweep_str(effective_sweep(o, dist));
    if (name == "sweep_set") return o.sweep_set ? "1" : "0";
    if (name == "split_tol") {
        char b[64];
        snprintf(b, sizeof b, "%.17g", o.split_tol);
        return b;
    }
    if (name == "batch") return std::to_string(o.batch);
    if (name == "r0_xcd_chunk") return std::to_string(o.r0_xcd_chunk);
    if (name == "chain_wide") return std::to_string(o.chain_wide);
    if (name == "fail_inject") return o.fail_inject;
    throw Error(CPK_ERR_ARGS, "unknown engine option '" + name + "'");
}

EngineOpts engine_opts_from_env() {
    EngineOpts o;
    auto from = [&](const char *name) {
        std::string env = "CPK_";
        for (const char *p = name; *p; p++) env += (char)toupper((unsigned char)*p);
        if (const char *e = getenv(env.c_str())) set_engine_option(o, name, e);
    };
    for (const BoolOpt &b : kBool) from(b.name);
    from("sweep");
    from("split_tol");
    from("batch");
    from("r0_xcd_chunk");
    from("chain_wide");
    from("fail_inject");
    return o;
}

std::string engine_opts_string(const EngineOpts &o, bool dist) {
    std::string s;
    auto put = [&](const std::string &name) { s += name + "=" + get_engine_option(o, name, dist) + ";"; };
    for (const BoolOpt &b : kBool) put(b.name);
    put("sweep");
    put("sweep_set");
    put("split_tol");
    put("batch");
    put("r0_xcd_chunk");
    put("chain_wide");
    put("fail_inject");
    return s;
}

void apply_engine_options(EngineOpts &o, const std::string &spec) {
    size_t p = 0;
    std::string sweep_set;
    while (p < spec.size()) {
        size_t q = spec.find(';', p);
        if (q == std::string::npos) q = spec.size();
        const std::string item = spec.substr(p, q - p);
        p = q + 1;
        if (item.empty()) continue;
        const size_t eq = item.find('=');
        if (eq == std::string::npos) throw Error(CPK_ERR_ARGS, "engine options: expected name=value, got '" + item + "'");
        const std::string name = item.substr(0, eq), value = item.substr(eq + 1);
        if (name == "sweep_set") sweep_set = value;  // after "sweep", whatever the order
        else set_engine_option(o, name, value);
    }
    if (!sweep_set.empty()) set_engine_option(o, "sweep_set", sweep_set);
}

uint64_t engine_opts_hash(const EngineOpts &o) {
    uint64_t h = 1469598103934665603ull;
    auto mix = [&](const std::string &s) {
        for (unsigned char ch : s) h = (h ^ ch) * 1099511628211ull;
        h = (h ^ 0xffu) * 1099511628211ull;
    };
    for (const BoolOpt &b : kBool) mix(b.name), mix(o.*b.m ? "1" : "0");
    mix(sweep_str(o.sweep));
    mix(o.sweep_set ? "1" : "0");
    mix(get_engine_option(o, "split_tol"));
    mix(std::to_string(o.batch));
    mix(std::to_string(o.r0_xcd_chunk));
    mix(std::to_string(o.chain_wide));
    // fail_inject is rank-local by design (a test hook): not hashed, so the plan agreement passes
    return h;
}

}  // namespace cpk
