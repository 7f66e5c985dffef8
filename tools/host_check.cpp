// Host-side sanitizer driver for libgnnd's graph builder (tools/host_sanitize.sh builds it
// with AddressSanitizer + UBSan on the host code only).  Builds the tables for random Tanner
// graphs of many shapes through gnnd_graph_validate_host (no device needed) and checks the
// structural invariants; exit 0 iff every graph is accepted and consistent, or rejected with
// the documented status (check degree > 256).
#include <cstdio>
#include <cstdint>
#include <random>
#include <vector>
#include "../include/gnnd.h"

int main(int argc, char** argv) {
    const int n = argc > 1 ? atoi(argv[1]) : 300;
    std::mt19937 rng(12345);
    int bad = 0, ok = 0, unsupported = 0;
    for (int t = 0; t < n; ++t) {
        const int V = 1 + rng() % 700, C = 1 + rng() % 400;
        const double dens = (t % 5 == 0) ? 0.5 : (1 + rng() % 12) / (double)C;
        std::vector<int64_t> var, chk;
        std::bernoulli_distribution b(dens > 1 ? 1 : dens);
        for (int v = 0; v < V; ++v)
            for (int c = 0; c < C; ++c)
                if (b(rng) && var.size() < 60000) { var.push_back(v); chk.push_back(c); }
        if (var.empty()) { var.push_back(0); chk.push_back(0); }
        int32_t rep[4] = {0, 0, 0, 0};
        const int rc = gnnd_graph_validate_host(var.data(), chk.data(), (int64_t)var.size(), V, C, rep);
        if (rc == GNND_OK && rep[3] == 0) ++ok;
        else if (rc == GNND_ERR_UNSUPPORTED) ++unsupported;
        else { ++bad; printf("graph %d (V=%d C=%d E=%zu): status %d, %d invariant failures\n", t, V, C, var.size(), rc, rep[3]); }
    }
    // malformed input is rejected, not read out of bounds
    int64_t v2[2] = {1, 0}, c2[2] = {0, 0};
    if (gnnd_graph_validate_host(v2, c2, 2, 2, 1, nullptr) != GNND_ERR_GRAPH) ++bad;
    int64_t v3[1] = {5}, c3[1] = {0};
    if (gnnd_graph_validate_host(v3, c3, 1, 2, 1, nullptr) != GNND_ERR_GRAPH) ++bad;
    printf("host_check: %d ok, %d unsupported, %d bad\n", ok, unsupported, bad);
    return bad ? 1 : 0;
}
