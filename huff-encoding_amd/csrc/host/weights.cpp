// weights.cpp — host half of ByteWeights (huff_coding/src/weights.rs).
// The counting pass itself is the hist256 GPU kernel (device/hist.hip).
#include "huff_coding.hpp"

namespace huff {

ByteWeights ByteWeights::from_counts(const uint64_t counts[256]) {
    ByteWeights bw;
    for (int b = 0; b < 256; ++b) {
        bw.weights[b] = counts[b];
        bw.len += counts[b] != 0;  // weights.rs:271 `if weights[b] == 0 { len += 1 }`
    }
    return bw;
}

size_t ByteWeights::iter(uint8_t letters[257], uint64_t w[257]) const {
    // Iter::next (weights.rs:423-441) scans an index 0..=256 and reads the
    // bin with `index as u8`; index 256 therefore aliases byte 0. The scan
    // stops at 256 unless byte 0 is non-zero there, which re-yields byte 0
    // exactly when the last non-zero bin is not 255.
    size_t count = 0;
    int last = -1;
    for (int b = 0; b < 256; ++b) {
        if (weights[b] != 0) {
            letters[count] = static_cast<uint8_t>(b);
            w[count] = weights[b];
            ++count;
            last = b;
        }
    }
    if (weights[0] != 0 && last != 255) {
        letters[count] = 0;
        w[count] = weights[0];
        ++count;
    }
    return count;
}

void ByteWeights::add(const ByteWeights& other) {
    uint8_t l[257];
    uint64_t f[257];
    size_t cnt = other.iter(l, f);
    for (size_t i = 0; i < cnt; ++i) {
        uint64_t& slot = weights[l[i]];
        if (slot != 0) {
            slot += f[i];       // weights.rs:379
        } else {
            slot = f[i];        // weights.rs:382-383
            len += 1;
        }
    }
}

std::vector<std::pair<size_t, size_t>> ration_bounds(size_t n, size_t ration_count) {
    // utils.rs:6-28: n / T per ration, the last takes the remainder; if
    // n / T == 0 the whole slice is a single ration.
    std::vector<std::pair<size_t, size_t>> r;
    size_t per = ration_count ? n / ration_count : 0;
    if (per == 0) {
        r.emplace_back(0, n);
        return r;
    }
    for (size_t i = 0; i < ration_count; ++i) {
        size_t b = i * per;
        size_t e = (i + 1 == ration_count) ? n : b + per;
        r.emplace_back(b, e);
    }
    return r;
}

ByteWeights shard_weights(const uint64_t* hists, uint32_t world) {
    ByteWeights g;
    for (uint32_t q = 0; q < world; ++q)
        for (int b = 0; b < 256; ++b) g.weights[b] += hists[static_cast<size_t>(q) * 256 + b];
    g.len = 0;
    for (int b = 0; b < 256; ++b) g.len += g.weights[b] != 0;
    return g;
}

uint64_t shard_bit_base(const uint64_t* hists, uint32_t rank, const uint8_t len[256]) {
    uint64_t base = 0;
    for (uint32_t q = 0; q < rank; ++q)
        for (int b = 0; b < 256; ++b) base += hists[static_cast<size_t>(q) * 256 + b] * len[b];
    return base;
}

void shard_prev_tail(const uint8_t* tails, const uint8_t* tail_lens, uint32_t rank, uint8_t prev[8], size_t* np) {
    size_t k = 0;
    for (uint32_t q = rank; q-- > 0 && k < 8;) {  // walk back over the earlier shards
        const size_t tl = tail_lens[q] > 8 ? 8 : tail_lens[q];
        for (size_t i = tl; i-- > 0 && k < 8;) prev[7 - k++] = tails[static_cast<size_t>(q) * 8 + i];
    }
    *np = k;
}

}  // namespace huff
