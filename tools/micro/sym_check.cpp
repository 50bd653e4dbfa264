// Checks the threaded symbolic LDL' (factor.cpp: ldl_symbolic_threaded, used with the device
// numeric phase) against the serial up-looking loop's structure on Kp / perm files written by
// tools/micro/sym_check.py: elimination tree, L's pattern, and every LdlSymbolic array.
#include <chrono>
#include <cstdio>
#include <fstream>
#include <vector>

#include "host.hpp"

using namespace cpk;

template <class T>
static std::vector<T> load(const char *path) {
    std::ifstream f(path, std::ios::binary | std::ios::ate);
    const size_t n = (size_t)f.tellg() / sizeof(T);
    std::vector<T> v(n);
    f.seekg(0);
    f.read(reinterpret_cast<char *>(v.data()), (std::streamsize)(n * sizeof(T)));
    return v;
}

int main(int argc, char **argv) {
    if (argc < 2) return 2;
    const std::string d = argv[1];
    HCsr Kp;
    Kp.ptr = load<int64_t>((d + "/ptr.bin").c_str());
    Kp.ind = load<int32_t>((d + "/ind.bin").c_str());
    Kp.val = load<double>((d + "/val.bin").c_str());
    Kp.nrows = Kp.ncols = (int64_t)Kp.ptr.size() - 1;
    const std::vector<int32_t> perm = load<int32_t>((d + "/perm.bin").c_str());
    LdlSymbolic a, b;
    auto t0 = std::chrono::steady_clock::now();
    const Factor fa = ldl_factor(Kp, perm, 1, &a, false);  // threaded symbolic
    auto t1 = std::chrono::steady_clock::now();
    const Factor fb = ldl_factor(Kp, perm, 1, &b, true);   // serial, with the numeric phase
    auto t2 = std::chrono::steady_clock::now();
    printf("threaded symbolic %.3f s, serial symbolic + numeric %.3f s\n", std::chrono::duration<double>(t1 - t0).count(),
           std::chrono::duration<double>(t2 - t1).count());
    int bad = 0;
    auto chk = [&](const char *what, bool ok) {
        if (!ok) printf("MISMATCH %s\n", what), bad++;
    };
    chk("parent", fa.parent == fb.parent);
    chk("Lp", fa.Lp == fb.Lp);
    chk("Li", fa.Li == fb.Li);
    chk("Rp", a.Rp == b.Rp);
    chk("Rc", a.Rc == b.Rc);
    chk("Rcsc", a.Rcsc == b.Rcsc);
    chk("kp_ptr", a.kp_ptr == b.kp_ptr);
    chk("kp_tgt", a.kp_tgt == b.kp_tgt);
    chk("kp_src", a.kp_src == b.kp_src);
    chk("lev_ptr", a.lev_ptr == b.lev_ptr);
    chk("lev_rows", a.lev_rows == b.lev_rows);
    printf("N %lld nnz(L) %zu: %s\n", (long long)Kp.nrows, fa.Li.size(), bad ? "MISMATCH" : "identical");
    return bad ? 1 : 0;
}
