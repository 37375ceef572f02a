// Host check of the snapshot builders' exact remainder (kad_dev.hpp mod_u64_u32: two fp64-reciprocal
// steps) against the integer %: edge dividends / divisors, then seeded random cases.  Exit 0 = equal.
#include "kad_dev.hpp"

#include <cstdio>
#include <cstdlib>
#include <random>

int main(int argc, char** argv)
{
    const long reps = argc > 1 ? atol(argv[1]) : 10000000;
    std::mt19937_64 g(0x5EEDull);
    unsigned long long bad = 0, n = 0;
    auto chk = [&](uint64_t h, uint32_t d) {
        ++n;
        if (ovs::mod_u64_u32(h, d) != (uint32_t)(h % d)) {
            if (bad < 5) printf("mismatch h=%llu d=%u\n", (unsigned long long)h, d);
            ++bad;
        }
    };
    const uint32_t ds[] = {1u, 2u, 3u, 7u, 1000003u, 1u << 24, (1u << 24) + 1, 0x7FFFFFFFu, 0x80000000u, 0xFFFFFFFEu,
                           0xFFFFFFFFu};
    const uint64_t hs[] = {0ull, 1ull, ~0ull, ~0ull - 1, 1ull << 63, (1ull << 53) - 1, 1ull << 53, (1ull << 43) - 1,
                           0x1FFFFFull, 0x1FFFFFull << 21};
    for (uint32_t d : ds)
        for (uint64_t h : hs) chk(h, d);
    for (long i = 0; i < reps; ++i) {
        const uint64_t h = g();
        uint32_t d = (uint32_t)(g() >> (32 + (g() & 31)));   // divisors spread over every magnitude
        if (!d) d = 1;
        chk(h, d);
        chk(~h, d);
        chk(h, 0xFFFFFFFFu - (uint32_t)(g() & 1023));
    }
    printf("checked %llu mismatches %llu\n", n, bad);
    return bad != 0;
}
