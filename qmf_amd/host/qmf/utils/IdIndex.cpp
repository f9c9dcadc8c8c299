#include <qmf/utils/IdIndex.h>

namespace qmf {

size_t IdIndex::getOrSetIdx(const int64_t id) {
  auto ins = idxMap_.emplace(id, ids_.size());
  if (ins.second) ids_.push_back(id);
  return ins.first->second;
}

void IdIndex::assignSorted(std::vector<int64_t> ids) {
  ids_ = std::move(ids);
  idxMap_.clear();
  idxMap_.reserve(ids_.size());
  for (size_t i = 0; i < ids_.size(); ++i) idxMap_.emplace(ids_[i], i);
}

}  // namespace qmf
