// FlatMap (opencv_amd/csrc/flat_map.hpp) against std::unordered_map: random
// insert / set / erase / find sequences at the loop's load, both key types;
// built and run by tests/test_host_sanitizers.py under ASan + UBSan.
#include <cstdio>
#include <cstdlib>
#include <random>
#include <unordered_map>

#include "flat_map.hpp"

template <class K>
static int check(unsigned seed, K span, size_t live_max)
{
    std::mt19937_64 rng(seed);
    tbdk::FlatMap<K> fm(4 * live_max);
    std::unordered_map<K, int> um;
    for (int op = 0; op < 200000; ++op) {
        const K k = (K)(rng() % span);
        const int v = (int)(rng() % 100000);
        switch (rng() % 4) {
        case 0:
            if (um.size() < live_max && fm.insert(k, v) != um.emplace(k, v).second) return 1;
            break;
        case 1:
            if (um.size() < live_max || um.count(k)) {
                fm.set(k, v);
                um[k] = v;
            }
            break;
        case 2:
            if (fm.erase(k) != (um.erase(k) > 0)) return 2;
            break;
        default: {
            const int* p = fm.find(k);
            auto it = um.find(k);
            if ((p != nullptr) != (it != um.end()) || (p && *p != it->second)) return 3;
        }
        }
        if (fm.size() != um.size()) return 4;
        if (op % 50000 == 49999) {  // per-step clear (the early-ROI table)
            fm.clear();
            um.clear();
        }
    }
    for (const auto& kv : um)
        if (!fm.find(kv.first) || *fm.find(kv.first) != kv.second) return 5;
    return 0;
}

// a table sized for far fewer entries than it receives grows instead of
// probing forever: 16 slots, 5000 live keys, then erase them all
static int check_growth()
{
    tbdk::FlatMap<unsigned> fm(16);
    for (unsigned k = 0; k < 5000; ++k) {
        if (!fm.insert(k * 7919u, (int)k)) return 6;
        fm.set(k * 7919u + 1u, -(int)k);
    }
    if (fm.size() != 10000 || fm.capacity() < 20000) return 7;
    for (unsigned k = 0; k < 5000; ++k) {
        const int* p = fm.find(k * 7919u);
        const int* q = fm.find(k * 7919u + 1u);
        if (!p || *p != (int)k || !q || *q != -(int)k) return 8;
    }
    for (unsigned k = 0; k < 5000; ++k)
        if (!fm.erase(k * 7919u) || !fm.erase(k * 7919u + 1u)) return 9;
    return fm.size() == 0 && !fm.find(7919u) ? 0 : 10;
}

int main()
{
    if (const int g = check_growth()) {
        std::printf("FAIL growth code %d\n", g);
        return 1;
    }
    for (unsigned s = 1; s <= 4; ++s) {
        int r = check<unsigned>(s, 600u, 256);  // track ids, dense collisions
        if (!r) r = check<unsigned long long>(s + 10, 1ull << 40, 1024);  // box keys, sparse
        if (r) {
            std::printf("FAIL seed %u code %d\n", s, r);
            return 1;
        }
    }
    std::printf("flat_map ok\n");
    return 0;
}
