// Checks transpose_pattern (hostsparse.cpp, the parallel CSC -> row transpose of the factor
// layout) against the serial column-by-column transpose on random strictly-lower patterns,
// empty rows and columns included, for several thread counts (CPK_THREADS).
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

#include "host.hpp"

using namespace cpk;

int main() {
    std::mt19937_64 rng(7);
    int bad = 0, cases = 0;
    for (int64_t N : {0, 1, 5, 100, 5000, 300000, 2000000}) {
        for (int dens : {0, 1, 3}) {
            std::vector<int64_t> Lp(N + 1, 0);
            std::vector<int32_t> Li;
            for (int64_t j = 0; j < N; j++) {
                const int64_t k = dens ? (int64_t)(rng() % (2 * dens + 1)) : 0;
                std::vector<int32_t> c;
                for (int64_t t = 0; t < k && j + 1 < N; t++) c.push_back((int32_t)(j + 1 + rng() % (N - j - 1)));
                std::sort(c.begin(), c.end());
                c.erase(std::unique(c.begin(), c.end()), c.end());
                Li.insert(Li.end(), c.begin(), c.end());
                Lp[j + 1] = (int64_t)Li.size();
            }
            const int64_t nnz = Lp[N];
            std::vector<uint32_t> rp(N + 1, 0), rp2(N + 1, 0);
            std::vector<int32_t> rc(nnz), ri(nnz), rc2(nnz), ri2(nnz);
            for (int32_t i : Li) rp2[i + 1]++;
            for (int64_t i = 0; i < N; i++) rp2[i + 1] += rp2[i];
            std::vector<uint32_t> nx(rp2.begin(), rp2.end() - 1);
            for (int64_t j = 0; j < N; j++)
                for (int64_t p = Lp[j]; p < Lp[j + 1]; p++) {
                    const uint32_t q = nx[Li[p]]++;
                    rc2[q] = (int32_t)j, ri2[q] = (int32_t)p;
                }
            for (const char *th : {"1", "3", "8", "16"}) {
                setenv("CPK_THREADS", th, 1);
                std::fill(rp.begin(), rp.end(), 7u);
                transpose_pattern(N, Lp.data(), Li.data(), rp.data(), rc.data(), ri.data());
                cases++;
                if (rp != rp2 || rc != rc2 || ri != ri2) {
                    printf("MISMATCH N %lld dens %d threads %s\n", (long long)N, dens, th);
                    bad++;
                }
            }
        }
    }
    printf("%d cases, %d mismatches\n", cases, bad);
    return bad != 0;
}
