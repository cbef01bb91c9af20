// flat_map.hpp — the TBD loop's per-frame lookup tables (track id -> slot,
// track id -> corner count, early-GFTT box -> row): open addressing with
// linear probing and backward-shift erase in arrays sized once for the loop's
// track capacity, so the frame's ~900 lookups and ~200 updates neither hash
// through std::hash's bucket division nor allocate a node per insert (an
// std::unordered_map version cost ~14 us of host time per 1080p x 128 frame,
// this one ~3.5 us, on the critical host chain of the frame).
#pragma once
#include <algorithm>
#include <cstddef>
#include <cstdint>
#include <vector>
namespace tbdk {

// K -> int; the capacity is a power of two, sized by the loop to 4x its
// track capacity.  An insert that would fill more than half of it doubles the
// table first (a rehash: pointers from find() do not survive an insert), so a
// load the sizing did not foresee costs a rehash instead of a probe that
// never meets an empty slot.
template <class K>
class FlatMap {
public:
    explicit FlatMap(size_t min_cap = 16)
    {
        size_t cap = 16;
        while (cap < min_cap) cap <<= 1;
        keys_.assign(cap, K());
        vals_.assign(cap, 0);
        used_.assign(cap, 0);
        mask_ = cap - 1;
    }
    int* find(K k)
    {
        for (size_t i = home(k);; i = (i + 1) & mask_) {
            if (!used_[i]) return nullptr;
            if (keys_[i] == k) return &vals_[i];
        }
    }
    // emplace semantics: false (value untouched) when k is present
    bool insert(K k, int v)
    {
        reserve_one();
        size_t i = home(k);
        for (; used_[i]; i = (i + 1) & mask_)
            if (keys_[i] == k) return false;
        keys_[i] = k;
        vals_[i] = v;
        used_[i] = 1;
        ++size_;
        return true;
    }
    void set(K k, int v)
    {
        reserve_one();
        size_t i = home(k);
        for (; used_[i]; i = (i + 1) & mask_)
            if (keys_[i] == k) {
                vals_[i] = v;
                return;
            }
        keys_[i] = k;
        vals_[i] = v;
        used_[i] = 1;
        ++size_;
    }
    bool erase(K k)
    {
        size_t i = home(k);
        for (;; i = (i + 1) & mask_) {
            if (!used_[i]) return false;
            if (keys_[i] == k) break;
        }
        // backward shift: pull later entries of the probe run into the hole
        for (size_t j = (i + 1) & mask_; used_[j]; j = (j + 1) & mask_) {
            const size_t h = home(keys_[j]);
            // entry j may move to hole i iff its home is not in the cyclic range (i, j]
            if (((j - h) & mask_) >= ((j - i) & mask_)) {
                keys_[i] = keys_[j];
                vals_[i] = vals_[j];
                i = j;
            }
        }
        used_[i] = 0;
        --size_;
        return true;
    }
    void clear()
    {
        if (size_) std::fill(used_.begin(), used_.end(), (uint8_t)0);
        size_ = 0;
    }
    size_t size() const { return size_; }
    size_t capacity() const { return mask_ + 1; }

private:
    void reserve_one()
    {
        if (2 * (size_ + 1) <= mask_ + 1) return;
        std::vector<K> ok;
        std::vector<int> ov;
        std::vector<uint8_t> ou;
        ok.swap(keys_);
        ov.swap(vals_);
        ou.swap(used_);
        const size_t cap = 2 * ok.size();
        keys_.assign(cap, K());
        vals_.assign(cap, 0);
        used_.assign(cap, 0);
        mask_ = cap - 1;
        for (size_t j = 0; j < ok.size(); ++j) {
            if (!ou[j]) continue;
            size_t i = home(ok[j]);
            while (used_[i]) i = (i + 1) & mask_;
            keys_[i] = ok[j];
            vals_[i] = ov[j];
            used_[i] = 1;
        }
    }
    size_t home(K k) const
    {
        uint64_t x = (uint64_t)k;
        x ^= x >> 33;
        x *= 0xff51afd7ed558ccdull;
        x ^= x >> 33;
        return (size_t)x & mask_;
    }
    std::vector<K> keys_;
    std::vector<int> vals_;
    std::vector<uint8_t> used_;
    size_t mask_ = 0, size_ = 0;
};

}  // namespace tbdk
