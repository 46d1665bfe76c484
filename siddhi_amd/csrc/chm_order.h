// Iteration order of the reference runtime's java.util.concurrent.ConcurrentHashMap (JDK 8), for
// the fan-out of a stream a partition does not key: PartitionStreamReceiver.send(ComplexEvent)
// (PartitionStreamReceiver.java:277-281) hands each event to every key's junction in the order of
// cachedStreamJunctionMap.values(), a map of "streamId + key" strings filled as keys are created
// (PartitionRuntime.updatePartitionStreamReceivers:312-316). The JDK is not part of the reference
// tree; this restates its published algorithm for a single-threaded map: putVal (bins of linked
// nodes, TreeBins past 8 nodes on tables of >= 64), addCount (resize at 3/4 load), transfer (split
// at the lastRun, earlier nodes prepended), tryPresize. Host code (engine.hip builds the per-key
// ranks the K_gen records carry).
#pragma once
#include <cstdint>
#include <string>
#include <vector>

namespace sdh {

// String.hashCode of prefix + s, from the prefix's hash (ASCII s: one UTF-16 unit per byte)
inline int32_t java_hash_cat(int32_t prefix_hash, const std::string& s) {
  uint32_t h = (uint32_t)prefix_hash;
  for (unsigned char c : s) h = h * 31u + c;
  return (int32_t)h;
}

// String.hashCode of prefix + s from s's own hashCode and UTF-16 length:
// h(p + s) = h(p) * 31^len(s) + h(s) (mod 2^32)
inline int32_t java_hash_cat_hashed(int32_t prefix_hash, int32_t s_hash, int64_t s_len) {
  uint32_t m = 1, b = 31;
  for (int64_t e = s_len; e > 0; e >>= 1) {
    if (e & 1) m *= b;
    b *= b;
  }
  return (int32_t)((uint32_t)prefix_hash * m + (uint32_t)s_hash);
}

// String.valueOf of a partition key's value (ValuePartitionExecutor.java:34-40): int / long in
// decimal, bool as true / false
inline std::string java_value_of(bool is_bool, int64_t v) {
  if (is_bool) return v ? "true" : "false";
  return std::to_string((long long)v);
}

// Keys inserted in order (their String.hashCode) -> their positions in the map's iteration order
class ChmOrder {
 public:
  std::vector<int32_t> positions(const std::vector<int32_t>& hashes) {
    const size_t n = hashes.size();
    spread_.resize(n);
    next_.assign(n, -1);
    head_.assign(16, -1);
    tree_.assign(16, 0);
    size_ctl_ = 12;
    for (size_t k = 0; k < n; ++k) put((int32_t)k, hashes[k], (int64_t)k + 1);
    std::vector<int32_t> pos(n, -1);
    int32_t r = 0;
    for (size_t b = 0; b < head_.size(); ++b)
      for (int32_t x = head_[b]; x >= 0; x = next_[x]) pos[(size_t)x] = r++;
    return pos;
  }

 private:
  std::vector<int32_t> spread_, next_, head_;
  std::vector<uint8_t> tree_;  // the bin is a TreeBin (its list is the TreeBin's `first` order)
  int64_t size_ctl_ = 0;

  void put(int32_t x, int32_t h, int64_t count_after) {
    const int32_t hs = (int32_t)(((uint32_t)h ^ ((uint32_t)h >> 16)) & 0x7fffffffu);
    spread_[(size_t)x] = hs;
    const size_t i = (size_t)hs & (head_.size() - 1);
    int64_t bin_count = 0;
    if (head_[i] < 0) {
      head_[i] = x;
    } else if (tree_[i]) {  // putTreeVal: the new TreeNode becomes `first`
      next_[(size_t)x] = head_[i];
      head_[i] = x;
      bin_count = 2;
    } else {  // appended at the tail; binCount = the nodes walked
      int32_t t = head_[i];
      bin_count = 1;
      while (next_[(size_t)t] >= 0) {
        t = next_[(size_t)t];
        ++bin_count;
      }
      next_[(size_t)t] = x;
      if (bin_count >= 8) {  // TREEIFY_THRESHOLD -> treeifyBin
        if (head_.size() < 64) presize((int64_t)head_.size() << 1);
        else tree_[i] = 1;
      }
    }
    (void)bin_count;
    while (count_after >= size_ctl_) transfer();
  }

  void presize(int64_t size) {  // tryPresize: grow until sizeCtl covers tableSizeFor(1.5 size + 1)
    int64_t c = 1;
    while (c < size + (size >> 1) + 1) c <<= 1;
    while (c > size_ctl_) transfer();
  }

  void transfer() {
    const size_t n = head_.size();
    std::vector<int32_t> nh(2 * n, -1);
    std::vector<uint8_t> nt(2 * n, 0);
    for (size_t i = 0; i < n; ++i) {
      const int32_t f = head_[i];
      if (f < 0) continue;
      int32_t lo = -1, hi = -1;
      if (!tree_[i]) {
        int32_t last = f;
        int bit = spread_[(size_t)f] & (int32_t)n;
        for (int32_t p = next_[(size_t)f]; p >= 0; p = next_[(size_t)p])
          if ((spread_[(size_t)p] & (int32_t)n) != bit) {
            bit = spread_[(size_t)p] & (int32_t)n;
            last = p;
          }
        (bit == 0 ? lo : hi) = last;  // the run keeps its links
        for (int32_t p = f; p != last;) {
          const int32_t q = next_[(size_t)p];
          int32_t& side = (spread_[(size_t)p] & (int32_t)n) == 0 ? lo : hi;
          next_[(size_t)p] = side;  // prepended
          side = p;
          p = q;
        }
      } else {  // TreeBin: split in `first` order; <= 6 nodes untreeify (UNTREEIFY_THRESHOLD)
        int32_t lt = -1, ht = -1, ln = 0, hn = 0;
        for (int32_t p = f; p >= 0;) {
          const int32_t q = next_[(size_t)p];
          next_[(size_t)p] = -1;
          if ((spread_[(size_t)p] & (int32_t)n) == 0) {
            (lt < 0 ? lo : next_[(size_t)lt]) = p;
            lt = p;
            ++ln;
          } else {
            (ht < 0 ? hi : next_[(size_t)ht]) = p;
            ht = p;
            ++hn;
          }
          p = q;
        }
        nt[i] = ln > 6;
        nt[i + n] = hn > 6;
      }
      nh[i] = lo;
      nh[i + n] = hi;
    }
    head_.swap(nh);
    tree_.swap(nt);
    size_ctl_ = (int64_t)(2 * n) - (int64_t)(n >> 1);
  }
};

}  // namespace sdh
