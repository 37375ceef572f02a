// ovs_ini.cpp -- OMNeT++ .ini subset parser binding the reference's parameter
// names to ovs_params (include/ovs_kbr.h).
//
// Semantics kept from OMNeT++ 4.x Cmdenv configuration:
//  * sections [General] and [Config <name>], `extends = A, B` chains,
//    lookup order: the named config, its extends chain (depth first), then
//    [General]; within a section the FIRST matching line wins;
//  * keys are module-path patterns: `*` matches within one path component,
//    `**` across components (e.g. `**.overlay*.chord.successorListSize`);
//  * values: numbers with units (s, ms, us, ns, B, KiB, MiB, MB, bps, Kbps,
//    Mbps, Gbps), true/false, quoted strings.  ${...} iterations are rejected.
// Parameters are resolved against the module paths of an OverSim
// SimpleUnderlayNetwork host (default.ini:1-30, 166-222, 383-433, 483, 540-560).
#include <cctype>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <string>
#include <vector>

#include "../../include/ovs_kbr.h"

namespace {

struct Entry {
    std::string key, value;
};
struct Section {
    std::vector<Entry> entries;
    std::vector<std::string> extends;
};

std::string trim(const std::string& s)
{
    size_t a = 0, b = s.size();
    while (a < b && std::isspace((unsigned char)s[a])) ++a;
    while (b > a && std::isspace((unsigned char)s[b - 1])) --b;
    return s.substr(a, b - a);
}

// OMNeT++ wildcard match: '*' = [^.]*, '**' = .*, '?' = one non-dot char
bool glob(const char* p, const char* s)
{
    while (*p) {
        if (p[0] == '*' && p[1] == '*') {
            p += 2;
            for (const char* t = s;; ++t) {
                if (glob(p, t)) return true;
                if (!*t) return false;
            }
        }
        if (*p == '*') {
            ++p;
            for (const char* t = s;; ++t) {
                if (glob(p, t)) return true;
                if (!*t || *t == '.') return false;
            }
        }
        if (*p == '?') {
            if (!*s || *s == '.') return false;
            ++p; ++s;
            continue;
        }
        if (*p != *s) return false;
        ++p; ++s;
    }
    return *s == 0;
}

bool parse_number(const std::string& v0, double* out, std::string* unit)
{
    std::string v = trim(v0);
    if (v.empty()) return false;
    char* end = nullptr;
    const double x = std::strtod(v.c_str(), &end);
    if (end == v.c_str()) return false;
    *unit = trim(std::string(end));
    *out = x;
    return true;
}

bool to_seconds(const std::string& v, double* out)
{
    double x; std::string u;
    if (!parse_number(v, &x, &u)) return false;
    if (u.empty() || u == "s") *out = x;
    else if (u == "ms") *out = x * 1e-3;
    else if (u == "us") *out = x * 1e-6;
    else if (u == "ns") *out = x * 1e-9;
    else if (u == "min") *out = x * 60;
    else return false;
    return true;
}

bool to_bytes(const std::string& v, double* out)
{
    double x; std::string u;
    if (!parse_number(v, &x, &u)) return false;
    if (u.empty() || u == "B") *out = x;
    else if (u == "KiB") *out = x * 1024;
    else if (u == "MiB") *out = x * 1024 * 1024;
    else if (u == "KB" || u == "kB") *out = x * 1000;
    else if (u == "MB") *out = x * 1e6;
    else if (u == "b") *out = x / 8;
    else return false;
    return true;
}

bool to_bps(const std::string& v, double* out)
{
    double x; std::string u;
    if (!parse_number(v, &x, &u)) return false;
    if (u.empty() || u == "bps") *out = x;
    else if (u == "Kbps" || u == "kbps") *out = x * 1e3;
    else if (u == "Mbps") *out = x * 1e6;
    else if (u == "Gbps") *out = x * 1e9;
    else return false;
    return true;
}

bool to_bool(const std::string& v, int32_t* out)
{
    const std::string t = trim(v);
    if (t == "true") { *out = 1; return true; }
    if (t == "false") { *out = 0; return true; }
    return false;
}

bool to_int(const std::string& v, int32_t* out)
{
    double x; std::string u;
    if (!parse_number(v, &x, &u) || !u.empty()) return false;
    *out = (int32_t)x;
    return true;
}

std::string unquote(const std::string& v)
{
    std::string t = trim(v);
    if (t.size() >= 2 && t.front() == '"' && t.back() == '"') return t.substr(1, t.size() - 2);
    return t;
}

}  // namespace

extern "C" ovs_status ovs_params_from_ini(ovs_params* p, const char* ini_text, const char* config_name, char* err,
                                          int err_len)
{
    auto set_err = [&](const std::string& m) {
        if (err && err_len > 0) std::snprintf(err, (size_t)err_len, "%s", m.c_str());
    };
    if (!p || !ini_text) { set_err("null argument"); return OVS_EINVAL; }
    std::map<std::string, Section> secs;
    std::string cur = "General";
    secs[cur];
    // parse (with backslash line continuation)
    std::string text(ini_text);
    size_t pos = 0;
    int lineno = 0;
    while (pos <= text.size()) {
        size_t nl = text.find('\n', pos);
        if (nl == std::string::npos) nl = text.size();
        std::string line = text.substr(pos, nl - pos);
        pos = nl + 1;
        ++lineno;
        while (!line.empty() && line.back() == '\\' && pos <= text.size()) {
            size_t nl2 = text.find('\n', pos);
            if (nl2 == std::string::npos) nl2 = text.size();
            line = line.substr(0, line.size() - 1) + text.substr(pos, nl2 - pos);
            pos = nl2 + 1;
            ++lineno;
        }
        // strip comment (not inside quotes)
        bool inq = false;
        for (size_t i = 0; i < line.size(); ++i) {
            if (line[i] == '"') inq = !inq;
            if (line[i] == '#' && !inq) { line = line.substr(0, i); break; }
        }
        line = trim(line);
        if (line.empty()) continue;
        if (line.front() == '[') {
            const size_t e = line.find(']');
            if (e == std::string::npos) { set_err("bad section header at line " + std::to_string(lineno)); return OVS_EINVAL; }
            std::string name = trim(line.substr(1, e - 1));
            if (name.rfind("Config ", 0) == 0) name = trim(name.substr(7));
            cur = name;
            secs[cur];
            continue;
        }
        const size_t eq = line.find('=');
        if (eq == std::string::npos) { set_err("expected key = value at line " + std::to_string(lineno)); return OVS_EINVAL; }
        const std::string k = trim(line.substr(0, eq)), v = trim(line.substr(eq + 1));
        if (k == "extends") {
            size_t a = 0;
            while (a <= v.size()) {
                size_t c = v.find(',', a);
                if (c == std::string::npos) c = v.size();
                const std::string nm = trim(v.substr(a, c - a));
                if (!nm.empty()) secs[cur].extends.push_back(nm);
                a = c + 1;
            }
            continue;
        }
        secs[cur].entries.push_back({k, v});
    }
    // section lookup order
    std::vector<std::string> order;
    std::vector<std::string> stack;
    if (config_name && *config_name && std::strcmp(config_name, "General") != 0) {
        if (!secs.count(config_name)) { set_err(std::string("no such config: ") + config_name); return OVS_EINVAL; }
        stack.push_back(config_name);
    }
    while (!stack.empty()) {
        const std::string s = stack.front();
        stack.erase(stack.begin());
        bool seen = false;
        for (auto& o : order) seen |= (o == s);
        if (seen) continue;
        if (!secs.count(s)) { set_err("extends unknown config: " + s); return OVS_EINVAL; }
        order.push_back(s);
        const auto& ex = secs[s].extends;
        stack.insert(stack.begin(), ex.begin(), ex.end());
    }
    order.push_back("General");

    std::string iter_key;
    auto lookup = [&](const std::string& path, std::string* val) -> bool {
        for (const auto& sname : order) {
            for (const auto& e : secs[sname].entries) {
                if (glob(e.key.c_str(), path.c_str())) {
                    *val = e.value;
                    if (e.value.find("${") != std::string::npos) iter_key = e.key;
                    return true;
                }
            }
        }
        return false;
    };

    const std::string ov = p->overlay == OVS_OVERLAY_KADEMLIA ? "kademlia"
                           : p->overlay == OVS_OVERLAY_KOORDE ? "koorde"
                           : p->overlay == OVS_OVERLAY_EPICHORD ? "epichord" : "chord";
    const std::string host = "SimpleUnderlayNetwork.overlayTerminal[0]";
    const std::string ovp = host + ".overlay." + ov + ".";
    std::string v, bad;

    auto want_int = [&](const std::string& name, int32_t* f) {
        if (lookup(ovp + name, &v) && !to_int(unquote(v), f)) bad = name;
    };
    auto want_bool = [&](const std::string& name, int32_t* f) {
        if (lookup(ovp + name, &v) && !to_bool(unquote(v), f)) bad = name;
    };
    want_int("keyLength", &p->keyLength);
    want_int("hopCountMax", &p->hopCountMax);
    if (p->overlay == OVS_OVERLAY_CHORD || p->overlay == OVS_OVERLAY_KOORDE) {
        want_int("successorListSize", &p->successorListSize);
        want_bool("extendedFingerTable", &p->extendedFingerTable);
        want_int("numFingerCandidates", &p->numFingerCandidates);
        if (p->overlay == OVS_OVERLAY_KOORDE) {   // Koorde.ned, default.ini:268-291
            want_int("shiftingBits", &p->shiftingBits);
            want_int("deBruijnListSize", &p->deBruijnListSize);
            want_bool("useOtherLookup", &p->useOtherLookup);
            want_bool("useSucList", &p->useSucList);
        }
    } else if (p->overlay == OVS_OVERLAY_EPICHORD) {   // EpiChord.ned, default.ini:145-164
        want_int("successorListSize", &p->successorListSize);
        if (lookup(ovp + "cacheTTL", &v) && !to_seconds(unquote(v), &p->cacheTTL)) bad = "cacheTTL";
    } else {
        want_int("k", &p->k);
        want_int("s", &p->s);
        want_int("b", &p->b);
        want_int("globalNodeLimit", &p->globalNodeLimit);
        want_int("extraNodesFinalBucket", &p->extraNodesFinalBucket);
        if (lookup(ovp + "bucketType", &v)) {
            // Kademlia::initializeOverlay (Kademlia.cc:135-151)
            const std::string bt = unquote(v);
            if (bt == "kademlia") p->bucketType = 0;
            else if (bt == "nkademlia") p->bucketType = 1;
            else if (bt == "nr128") p->bucketType = 2;
            else bad = "bucketType";
        }
    }
    want_int("lookupRedundantNodes", &p->lookupRedundantNodes);
    want_int("lookupParallelPaths", &p->lookupParallelPaths);
    want_int("lookupParallelRpcs", &p->lookupParallelRpcs);
    want_bool("lookupMerge", &p->lookupMerge);
    want_bool("lookupStrictParallelRpcs", &p->lookupStrictParallelRpcs);
    want_bool("lookupVisitOnlyOnce", &p->lookupVisitOnlyOnce);
    want_bool("lookupAcceptLateSiblings", &p->lookupAcceptLateSiblings);
    want_bool("lookupUseAllParallelResponses", &p->lookupUseAllParallelResponses);
    want_bool("lookupNewRpcOnEveryTimeout", &p->lookupNewRpcOnEveryTimeout);
    want_bool("lookupNewRpcOnEveryResponse", &p->lookupNewRpcOnEveryResponse);
    want_bool("lookupFinishOnFirstUnchanged", &p->lookupFinishOnFirstUnchanged);
    want_bool("lookupVerifySiblings", &p->lookupVerifySiblings);
    want_bool("lookupMajoritySiblings", &p->lookupMajoritySiblings);
    want_int("recNumRedundantNodes", &p->recNumRedundantNodes);
    // route-message options that change the recursive message format: only their defaults
    for (const char* opt : {"recordRoute", "routeMsgAcks"}) {
        int32_t on = 0;
        if (lookup(ovp + opt, &v)) {
            if (!to_bool(unquote(v), &on)) bad = opt;
            else if (on) {
                set_err(std::string(opt) + " = true not supported (default.ini:398,434 set false)");
                return OVS_ENOTSUP;
            }
        }
    }
    if (lookup(ovp + "routingType", &v)) {
        const std::string rt = unquote(v);
        // BaseOverlay::initialize routingType names (BaseOverlay.cc:119-131)
        if (rt == "iterative") p->routingType = 0;
        else if (rt == "semi-recursive") p->routingType = 1;
        else if (rt == "full-recursive") p->routingType = 2;
        else if (rt == "exhaustive-iterative") p->routingType = 3;
        else if (rt == "source-routing-recursive") p->routingType = 4;
        else {
            set_err("routingType \"" + rt + "\" not supported (iterative, semi-recursive, full-recursive, "
                    "exhaustive-iterative, source-routing-recursive)");
            return OVS_ENOTSUP;
        }
    }
    if (lookup(ovp + "rpcUdpTimeout", &v) && !to_seconds(unquote(v), &p->rpcUdpTimeout)) bad = "rpcUdpTimeout";
    if (lookup(ovp + "rpcKeyTimeout", &v) && !to_seconds(unquote(v), &p->rpcKeyTimeout)) bad = "rpcKeyTimeout";
    const std::string udp = host + ".udp.";
    if (lookup(udp + "jitter", &v)) {
        double x; std::string u;
        if (!parse_number(unquote(v), &x, &u) || !u.empty()) bad = "jitter"; else p->jitter = x;
    }
    if (lookup(udp + "useCoordinateBasedDelay", &v) && !to_bool(unquote(v), &p->useCoordinateBasedDelay))
        bad = "useCoordinateBasedDelay";
    if (lookup(udp + "constantDelay", &v) && !to_seconds(unquote(v), &p->constantDelay)) bad = "constantDelay";
    const std::string app = host + ".tier1.kbrTestApp.";
    if (lookup(app + "testMsgSize", &v)) {
        double b;
        if (!to_bytes(unquote(v), &b)) bad = "testMsgSize"; else p->testMsgSize = (int32_t)b;
    }
    // SimpleUnderlay channel of every terminal (SimpleUnderlayConfigurator: churnGenerator channelTypes,
    // default.ini:559-562; channels.ned): one lossless type binds datarate and the access delay
    const std::string churn = "SimpleUnderlayNetwork.churnGenerator[0].";
    if (lookup(churn + "channelTypes", &v)) {
        const std::string ct = trim(unquote(v));
        if (ct.find(' ') != std::string::npos) {
            set_err("channelTypes \"" + ct + "\": several channel types give nodes different datarates and "
                    "access delays; the engine holds one channel for all nodes");
            return OVS_ENOTSUP;
        }
        if (ct == "oversim.common.simple_ethernetline") { p->datarate = 10e6; p->accessDelay = 0.0; }
        else if (ct == "oversim.common.simple_dsl") { p->datarate = 1e6; p->accessDelay = 0.020; }
        else if (!ct.empty()) {
            set_err("channelTypes \"" + ct + "\" not supported (simple_ethernetline, simple_dsl; the lossy "
                    "channels drop packets at random, channels.ned:11-35)");
            return OVS_ENOTSUP;
        }
    }
    if (lookup(churn + "channelTypesRx", &v) && !trim(unquote(v)).empty()) {
        set_err("channelTypesRx \"" + unquote(v) + "\": separate receive channels are not modelled");
        return OVS_ENOTSUP;
    }
    // channel parameters (channels.ned defaults unless overridden as ovs.datarate/ovs.accessDelay)
    if (lookup("ovs.datarate", &v) && !to_bps(unquote(v), &p->datarate)) bad = "datarate";
    if (lookup("ovs.accessDelay", &v) && !to_seconds(unquote(v), &p->accessDelay)) bad = "accessDelay";
    if (lookup("ovs.simtimeRounding", &v)) {
        const std::string r = unquote(v);
        if (r == "round") p->simtimeRound = 1;
        else if (r == "truncate") p->simtimeRound = 0;
        else bad = "simtimeRounding";
    }
    want_bool("measureAuthBlock", &p->measureAuthBlock);   // BaseOverlay.cc:113, CommonMessages.msg:57, 73
    if (!bad.empty()) { set_err("cannot parse value of " + bad + ": " + v); return OVS_EINVAL; }

    // Keys the engine does not model but that change a route, a response size or a delay.  A
    // stock config that sets one gets OVS_ENOTSUP naming the key, never a silently different
    // result.  The default.ini values pass.
    auto is_true = [&](const std::string& path, const char* name, bool* on) -> bool {
        int32_t b = 0;
        *on = false;
        if (!lookup(path, &v)) return true;
        if (!to_bool(unquote(v), &b)) { set_err(std::string("cannot parse value of ") + name + ": " + v); return false; }
        *on = b != 0;
        return true;
    };
    auto refuse = [&](const std::string& m) { set_err(m); return OVS_ENOTSUP; };
    auto study = [&]() { return v.find("${") != std::string::npos; };   // reported below, by key
    bool on = false;
    // the network and its clock: SimpleUnderlayNetwork (the delay model restated), simtime-scale -9
    // (int64 ns, default.ini:16, 27)
    if (lookup("network", &v) && !study() && unquote(v) != "oversim.underlay.simpleunderlay.SimpleUnderlayNetwork")
        return refuse("network = " + unquote(v) + " not supported: the engine restates SimpleUnderlay's delay "
                      "model (SimpleNodeEntry.cc:155-195)");
    if (lookup("simtime-scale", &v) && !study() && trim(v) != "-9")
        return refuse("simtime-scale = " + trim(v) + " not supported: latencies are int64 ns (simtime-scale = -9)");
    // overlayType (default.ini:624) must name the overlay these parameters are for
    if (lookup(host + ".overlayType", &v) && !study()) {
        std::string mod = unquote(v);
        mod = mod.substr(mod.rfind('.') == std::string::npos ? 0 : mod.rfind('.') + 1);
        const int32_t want = mod == "ChordModules" ? OVS_OVERLAY_CHORD : mod == "KademliaModules" ? OVS_OVERLAY_KADEMLIA
                             : mod == "KoordeModules" ? OVS_OVERLAY_KOORDE : mod == "EpiChordModules" ? OVS_OVERLAY_EPICHORD
                                                                                                      : -1;
        if (want < 0)
            return refuse("overlayType = " + unquote(v) + " not supported: the engine routes Chord, Kademlia, Koorde "
                          "and EpiChord");
        if (want != p->overlay) {
            set_err("overlayType = " + unquote(v) + " but the parameters are bound for " + ov);
            return OVS_EINVAL;
        }
    }
    // BaseRpc::sendRpcCall (BaseRpc.cc:197-200): the timeout becomes NeighborCache::getNodeTimeout
    // (RTT history or NCS estimate, NeighborCache.cc:802-850) -- entries are recorded from every
    // response whether or not enableNeighborCache is set (BaseRpc.cc:455-461, NeighborCache.cc:229, 282)
    if (!is_true(ovp + "optimizeTimeouts", "optimizeTimeouts", &on)) return OVS_EINVAL;
    if (on) return refuse("optimizeTimeouts = true not supported: RPC timeouts from NeighborCache::getNodeTimeout "
                          "(BaseRpc.cc:197-200) replace rpcUdpTimeout");
    // SimpleUDP::initialize (SimpleUDP.cc:128-142): a known fault type adds a hashed error to every
    // coordinate delay (SimpleNodeEntry.cc:188, 197-254); any other string is "no fault"
    if (lookup(host + ".udp.delayFaultType", &v)) {
        const std::string f = unquote(v);
        if (f == "live_all" || f == "live_planetlab" || f == "simulation")
            return refuse("udp.delayFaultType = \"" + f + "\" not supported: faulty coordinate delays "
                          "(SimpleNodeEntry.cc:197-254)");
    }
    // BaseRpc::internalSendRpcResponse (BaseRpc.cc:543-550): with an NCS every response carries the
    // node's coordinates (BASERESPONSE_L, CommonMessages.msg:73-76), which changes its length
    const std::string nc = host + ".neighborCache.";
    if (lookup(nc + "ncsType", &v) && unquote(v) != "none") {
        const std::string ncs = unquote(v);
        if (!is_true(nc + "ncsSendBackOwnCoords", "ncsSendBackOwnCoords", &on)) return OVS_EINVAL;
        if (on || !lookup(nc + "ncsSendBackOwnCoords", &v))   // NeighborCache.ned default: true
            return refuse("neighborCache.ncsType = \"" + ncs + "\" not supported: responses carry NcsInfo "
                          "(BaseRpc.cc:543-550), which changes their size");
    }
    // malicious nodes answer FindNodeCalls with the configured attacks (BaseOverlay.cc:1844-1907)
    const std::string gnl = "SimpleUnderlayNetwork.globalObserver.globalNodeList.";
    if (lookup(gnl + "maliciousNodeProbability", &v)) {
        double x; std::string u;
        if (!parse_number(unquote(v), &x, &u) || !u.empty()) { set_err("cannot parse value of maliciousNodeProbability: " + v); return OVS_EINVAL; }
        if (x > 0) return refuse("maliciousNodeProbability > 0 not supported: malicious nodes (GlobalNodeList.cc:221, "
                                 "BaseOverlay.cc:1844-1907)");
    }
    if (!is_true(gnl + "maliciousNodeChange", "maliciousNodeChange", &on)) return OVS_EINVAL;
    if (on) return refuse("maliciousNodeChange = true not supported: malicious nodes (GlobalNodeList.cc:79-80)");
    const bool recursive = p->routingType == 1 || p->routingType == 2 || p->routingType == 4;
    if (p->overlay == OVS_OVERLAY_KADEMLIA) {
        // R/Kademlia: findNode ranks route-message next hops by proximity (Kademlia.cc:1144-1157,
        // 1234-1241); with iterative routing every findNode serves a FindNodeCall and it has no effect
        if (!is_true(ovp + "proximityRouting", "proximityRouting", &on)) return OVS_EINVAL;
        if (on && recursive)
            return refuse("kademlia.proximityRouting = true not supported with recursive routing: findNode "
                          "orders route-message hops by proximity (Kademlia.cc:1144-1157, 1234-1241)");
        // altRecMode sets recordRoute (Kademlia.cc:133) and changes recursiveRoutingHook (1029-1063)
        if (!is_true(ovp + "altRecMode", "altRecMode", &on)) return OVS_EINVAL;
        if (on) return refuse("kademlia.altRecMode = true not supported: it sets recordRoute (Kademlia.cc:133) and "
                              "changes recursiveRoutingHook (Kademlia.cc:1029-1063)");
        // Kademlia::routingAdd options: the maintenance rounds (ovs_kad_maintenance_round) restate
        // routingAdd with them off, and the tables they converge to differ
        static const struct { const char* key; const char* where; } radd[] = {
            {"proximityNeighborSelection", "Kademlia.cc:682-756"},
            {"enableManagedConnections", "Kademlia.cc:660, 698, 720"},
            {"activePing", "Kademlia.cc:447, 682"},
            {"secureMaintenance", "Kademlia.cc:284, 459-489, 539-729"},
            {"pingNewSiblings", "Kademlia.cc:553"},
        };
        for (const auto& r : radd) {
            if (!is_true(ovp + r.key, r.key, &on)) return OVS_EINVAL;
            if (on)
                return refuse(std::string("kademlia.") + r.key + " = true not supported: it changes "
                              "Kademlia::routingAdd (" + r.where + "), which the maintenance rounds restate with it off");
        }
    }
    if (p->overlay == OVS_OVERLAY_CHORD && p->extendedFingerTable) {
        // handleRpcFixfingersResponse re-ranks a finger's candidates by measured proximity (Chord.cc:1290-1314)
        if (!is_true(ovp + "proximityRouting", "proximityRouting", &on)) return OVS_EINVAL;
        if (on)
            return refuse("chord.proximityRouting = true not supported with extendedFingerTable: finger candidates "
                          "ordered by proximity (Chord.cc:1290-1314)");
    }
    if (!iter_key.empty()) {
        set_err("parameter studies (${...}) are not supported: " + iter_key);
        return OVS_ENOTSUP;
    }
    return OVS_OK;
}

// OMNeT++ `include <file>` lines are textual inclusion relative to the including file
// (omnetpp.ini:520 `include ./default.ini`); resolved recursively, depth-limited against cycles.
static bool read_ini_file(const std::string& path, int depth, std::string* out, std::string* err)
{
    if (depth > 16) { *err = "include nesting too deep at " + path; return false; }
    std::FILE* f = std::fopen(path.c_str(), "rb");
    if (!f) { *err = "cannot open " + path; return false; }
    std::string text;
    char buf[65536];
    size_t got;
    while ((got = std::fread(buf, 1, sizeof buf, f)) > 0) text.append(buf, got);
    std::fclose(f);
    const size_t slash = path.rfind('/');
    const std::string dir = slash == std::string::npos ? std::string() : path.substr(0, slash + 1);
    size_t pos = 0;
    while (pos <= text.size()) {
        size_t nl = text.find('\n', pos);
        if (nl == std::string::npos) nl = text.size();
        const std::string raw = text.substr(pos, nl - pos), line = trim(raw);
        pos = nl + 1;
        if (line.rfind("include", 0) == 0 && line.size() > 7 && std::isspace((unsigned char)line[7])) {
            std::string inc = trim(line.substr(8));
            if (inc.empty()) { *err = "empty include in " + path; return false; }
            if (inc[0] != '/') inc = dir + inc;
            if (!read_ini_file(inc, depth + 1, out, err)) return false;
            out->push_back('\n');
        } else {
            out->append(raw);
            out->push_back('\n');
        }
    }
    return true;
}

extern "C" ovs_status ovs_params_from_ini_file(ovs_params* p, const char* path, const char* config_name, char* err,
                                               int err_len)
{
    if (!p || !path) {
        if (err && err_len > 0) std::snprintf(err, (size_t)err_len, "null argument");
        return OVS_EINVAL;
    }
    std::string text, e;
    if (!read_ini_file(path, 0, &text, &e)) {
        if (err && err_len > 0) std::snprintf(err, (size_t)err_len, "%s", e.c_str());
        return OVS_EINVAL;
    }
    return ovs_params_from_ini(p, text.c_str(), config_name, err, err_len);
}

// defaults = the reference's default.ini values (host-only parameter handling, with the binder above)
extern "C" void ovs_params_default(int32_t overlay, ovs_params* p)
{
    std::memset(p, 0, sizeof *p);
    p->overlay = overlay;
    p->keyLength = 160;                 // default.ini:393
    p->hopCountMax = 50;                // default.ini:385
    p->successorListSize = 8;           // default.ini:174
    p->extendedFingerTable = 0;         // default.ini:176
    p->numFingerCandidates = 3;         // default.ini:177
    p->k = 8; p->s = 8; p->b = 1;       // default.ini:197-199
    p->lookupParallelPaths = 1;
    p->lookupStrictParallelRpcs = 1;    // default.ini:425-433
    p->lookupVisitOnlyOnce = 1;
    p->lookupAcceptLateSiblings = 1;
    p->numSiblings = 1;                 // BaseOverlay::route -> sendToKey(..., 1, ...) (BaseOverlay.cc:1357)
    p->useCoordinateBasedDelay = 1;     // default.ini:546
    p->simtimeRound = 1;
    p->testMsgSize = 100;               // default.ini:37
    p->recNumRedundantNodes = 3;        // default.ini:386
    p->rpcUdpTimeout = 1.5;             // default.ini:483
    p->lookupTimeout = 10.0;            // IterativeLookup.h:44
    p->jitter = 0.0;                    // default.ini:549 has 0.1; bit-exact latency needs 0
    p->constantDelay = 0.05;            // default.ini:544
    p->datarate = 10e6;                 // channels.ned simple_ethernetline
    p->accessDelay = 0.0;
    p->kadSeed = 0x4b41444dull;
    p->shiftingBits = 4;                // default.ini:277
    p->deBruijnListSize = 16;           // default.ini:276
    p->useOtherLookup = 1;              // default.ini:279
    p->useSucList = 1;                  // default.ini:280
    p->cacheTTL = 120.0;                // default.ini:158
    p->bucketType = 0;                  // default.ini:209 "kademlia"
    p->globalNodeLimit = 1000;          // default.ini:210
    p->extraNodesFinalBucket = 0;       // default.ini:211
    p->rpcKeyTimeout = 10.0;            // default.ini:484
    p->measureAuthBlock = 0;            // default.ini:399
    if (overlay == OVS_OVERLAY_KOORDE) p->successorListSize = 16;   // default.ini:275
    if (overlay == OVS_OVERLAY_EPICHORD) p->successorListSize = 4;  // default.ini:159
    if (overlay == OVS_OVERLAY_KADEMLIA) {
        p->lookupRedundantNodes = 8;    // default.ini:186
        p->lookupParallelRpcs = 3;      // default.ini:188
        p->lookupMerge = 1;             // default.ini:189
    } else if (overlay == OVS_OVERLAY_EPICHORD) {
        p->lookupRedundantNodes = 3;    // default.ini:146
        p->lookupParallelRpcs = 1;      // default.ini:148
        p->lookupMerge = 1;             // default.ini:149
    } else {
        p->lookupRedundantNodes = 1;    // default.ini:423
        p->lookupParallelRpcs = 1;      // default.ini:425
        p->lookupMerge = 0;             // default.ini:428
    }
}
