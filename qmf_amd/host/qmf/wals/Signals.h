// Interaction grouping for WALS (reference: WALSEngine::groupSignals / sortDataset,
// qmf/wals/WALSEngine.cpp:130-163, and IdIndex).  The reference sorts the dataset by
// (userId, itemId), assigns user idx in ascending-id order, groups each user's signals in
// ascending item-id order, then repeats with the roles swapped.  This builds the same two
// CSR matrices directly: idx = rank of the id among the distinct ids, rows in idx order,
// each row's entries in ascending column idx (= ascending id), duplicates of a (u, i) pair
// kept, in input order.  Column indices are idx of the other side, 32-bit.
#pragma once

#include <cstdint>
#include <vector>

#include <qmf/DatasetReader.h>
#include <qmf/Types.h>
#include <qmf/utils/IdIndex.h>

namespace qmf {

struct SignalCsr {
  std::vector<int64_t> rowptr;  // nrows + 1
  std::vector<int32_t> col;     // nnz, idx on the other side
  std::vector<Double> val;      // nnz
  size_t nrows() const { return rowptr.empty() ? 0 : rowptr.size() - 1; }
  size_t nnz() const { return col.size(); }
};

// Builds userIndex / itemIndex (ascending ids) and both orientations.
void groupSignals(const std::vector<DatasetElem>& dataset, IdIndex& userIndex,
                  IdIndex& itemIndex, SignalCsr& byUser, SignalCsr& byItem, size_t nthreads);

// Sorted distinct values of `ids` (parallel chunk sort + merge).
std::vector<int64_t> sortedUnique(std::vector<int64_t> ids, size_t nthreads);

}  // namespace qmf
