// Raw id <-> contiguous idx mapping (reference: qmf/utils/IdIndex.h:27-62, IdIndex.cpp:21-31).
// BPR assigns idx in first-appearance order through getOrSetIdx; WALS builds the index in
// one shot from the ascending unique ids (assignSorted), which is the order the reference's
// sort-then-getOrSetIdx produces (WALSEngine.cpp:130-163).
#pragma once

#include <cstddef>
#include <cstdint>
#include <limits>
#include <unordered_map>
#include <vector>

namespace qmf {

class IdIndex {
 public:
  static const size_t missingIdx = std::numeric_limits<size_t>::max();

  IdIndex() = default;

  int64_t id(const size_t idx) const { return ids_[idx]; }

  size_t idx(const int64_t id) const {
    const auto it = idxMap_.find(id);
    return it == idxMap_.end() ? missingIdx : it->second;
  }

  // idx of `id`, appending a new entry when absent
  size_t getOrSetIdx(const int64_t id);

  // replaces the index with `ids` (must be unique); idx i <-> ids[i]
  void assignSorted(std::vector<int64_t> ids);

  size_t size() const { return ids_.size(); }
  const std::vector<int64_t>& ids() const { return ids_; }

  void reset() {
    ids_.clear();
    idxMap_.clear();
  }

 private:
  std::vector<int64_t> ids_;
  std::unordered_map<int64_t, size_t> idxMap_;
};

}  // namespace qmf
