// sanitize_driver.cpp -- exercises the CPU oracle (oracle/ovs_oracle.c) and the host-side
// .ini binder (oversim_amd/csrc/ovs_ini.cpp) under AddressSanitizer + UndefinedBehaviorSanitizer
// (tests/test_sanitizers.py builds it with -Wall -Wextra -Werror and runs it).  Test
// infrastructure only: small seeded networks, every entry point once, exit 0 when clean.
#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "../include/ovs_kbr.h"
#include "../oracle/ovs_oracle.h"

namespace {

uint64_t g_rng = 0x9E3779B97F4A7C15ull;
uint32_t rnd32()
{
    g_rng ^= g_rng << 13; g_rng ^= g_rng >> 7; g_rng ^= g_rng << 17;
    return (uint32_t)(g_rng >> 16);
}

bool key_less(const orc_key& a, const orc_key& b)
{
    for (int i = 4; i >= 0; --i)
        if (a.w[i] != b.w[i]) return a.w[i] < b.w[i];
    return false;
}

struct Net {
    std::vector<orc_key> ids;
    std::vector<double> xy;
};

Net population(uint32_t n)
{
    Net net;
    while (net.ids.size() < n) {
        orc_key k;
        for (auto& w : k.w) w = rnd32();
        net.ids.push_back(k);
        if (net.ids.size() == n) {
            std::sort(net.ids.begin(), net.ids.end(), key_less);
            net.ids.erase(std::unique(net.ids.begin(), net.ids.end(),
                                      [](const orc_key& a, const orc_key& b) { return !key_less(a, b) && !key_less(b, a); }),
                          net.ids.end());
        }
    }
    for (uint32_t i = 0; i < 2 * n; ++i) net.xy.push_back((double)(rnd32() % 150000) / 1000.0 - 75.0);
    return net;
}

int fails = 0;
void check(bool ok, const char* what)
{
    if (!ok) { std::fprintf(stderr, "FAIL: %s (%s)\n", what, orc_last_error()); ++fails; }
}

void route_some(orc_net* net, const Net& p, int numSiblings)
{
    const uint32_t m = 300, n = (uint32_t)p.ids.size();
    std::vector<orc_key> keys(m);
    std::vector<uint32_t> src(m), hop(m * 50), rpcs(m), sib(m * 16);
    std::vector<orc_route_out> out(m);
    std::vector<orc_lookup_out> lout(m);
    for (uint32_t i = 0; i < m; ++i) {
        keys[i] = (i & 1) ? p.ids[rnd32() % n] : orc_key{{rnd32(), rnd32(), rnd32(), rnd32(), rnd32()}};
        src[i] = rnd32() % n;
    }
    check(orc_route_batch(net, keys.data(), src.data(), m, out.data(), hop.data(), rpcs.data(), 2) != ORC_FAIL,
          "route batch");
    check(orc_lookup_batch(net, keys.data(), src.data(), m, numSiblings, lout.data(), sib.data(), 2) >= 0,
          "lookup batch");
    orc_kbrtest_result st;
    orc_kbrtest_stats(net, out.data(), keys.data(), src.data(), m, 30.0, 1, 100, &st);
    orc_kbrtest_lookup_result ls;
    orc_kbrtest_lookup_stats(net, lout.data(), sib.data(), numSiblings, keys.data(), src.data(), m, 30.0, 1, 10.0,
                             &ls);
    uint32_t nodes[64];
    int flag = 0;
    check(orc_find_node(net, src[0], &keys[0], 8, 1, nodes, &flag) >= 0, "find node");
}

}  // namespace

int main()
{
    // ---- oracle: Chord (stored, lazy, explicit tables + a fixfingers round), Kademlia (stored, lazy)
    for (uint32_t n : {2u, 9u, 700u}) {
        Net p = population(n);
        orc_params cp;
        orc_params_chord_default(&cp);
        for (int lazy = 0; lazy < 2; ++lazy) {
            orc_net* net = lazy ? orc_chord_build_lazy(p.ids.data(), n, p.xy.data(), &cp)
                                : orc_chord_build(p.ids.data(), n, p.xy.data(), &cp);
            check(net != nullptr, "chord build");
            route_some(net, p, 3 < (int)n - 1 ? 3 : 1);
            std::vector<uint32_t> f((size_t)n * 160);
            orc_chord_export_fingers(net, f.data());
            uint64_t ok = 0, ch = 0;
            std::vector<uint32_t> all(n);
            for (uint32_t i = 0; i < n; ++i) all[i] = i;
            orc_chord_fix_fingers(net, all.data(), n, &ok, &ch, 2);
            orc_net_free(net);
        }
        orc_params kp;
        orc_params_kad_default(&kp);
        for (int lazy = 0; lazy < 2; ++lazy) {
            orc_net* net = lazy ? orc_kad_build_lazy(p.ids.data(), n, p.xy.data(), &kp)
                                : orc_kad_build(p.ids.data(), n, p.xy.data(), &kp);
            check(net != nullptr, "kad build");
            route_some(net, p, 8);
            std::vector<uint32_t> sib((size_t)n * 40), bn((size_t)n * 160 * 8);
            std::vector<uint8_t> bc((size_t)n * 160);
            orc_kad_export(net, sib.data(), bc.data(), bn.data());
            orc_net_free(net);
        }
        kp.lookupParallelRpcs = 1;
        kp.rpcUdpTimeout = 0.3;           // RPC timeouts, dead nodes
        orc_net* net = orc_kad_build(p.ids.data(), n, p.xy.data(), &kp);
        route_some(net, p, 8);
        orc_net_free(net);
    }
    // ---- host .ini binder (oversim_amd/csrc/ovs_ini.cpp)
    ovs_params P;
    ovs_params_default(OVS_OVERLAY_CHORD, &P);
    char err[256];
    const char* ini =
        "[General]\n**.overlay*.chord.successorListSize = 4\n**.hopCountMax = 20\n**.rpcUdpTimeout = 1500ms\n"
        "[Config X]\nextends = General\n**.overlay*.*.lookupParallelRpcs = 2\n**.udp.jitter = 0\n";
    check(ovs_params_from_ini(&P, ini, "X", err, sizeof err) == OVS_OK, "ini parse");
    check(P.successorListSize == 4 && P.hopCountMax == 20 && P.lookupParallelRpcs == 2, "ini values");
    check(ovs_params_from_ini(&P, "[Config Y]\nextends = Nope\n", "Y", err, sizeof err) != OVS_OK, "ini error path");
    std::printf("sanitize driver: %s\n", fails ? "FAILED" : "clean");
    return fails ? 1 : 0;
}
