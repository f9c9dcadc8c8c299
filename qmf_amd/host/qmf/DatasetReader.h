// Dataset text reader (reference: qmf/DatasetReader.h:29-58, DatasetReader.cpp:29-59).
// Each line is "<userId> <itemId> <value>" parsed with sscanf("%lld %lld %lf") semantics;
// a malformed line aborts with "the file format is incorrect: <line>".  readAll() on a file
// parses fixed-size chunks on all host threads; the result is
// identical to the sequential readOne() loop.
#pragma once

#include <cstdint>
#include <istream>
#include <memory>
#include <string>
#include <vector>

#include <qmf/Types.h>

namespace qmf {

struct DatasetElem {
  int64_t userId;
  int64_t itemId;
  Double value = 1.0;
} __attribute__((aligned(1), __packed__));

static_assert(sizeof(DatasetElem) == 24, "DatasetElem must stay 24 bytes packed");

class DatasetReader {
 public:
  DatasetReader() = default;
  explicit DatasetReader(const std::string& fileName);
  // reads from an arbitrary stream (tests, pipes)
  explicit DatasetReader(std::unique_ptr<std::istream> stream);

  // reads one line; false at end of input
  bool readOne(DatasetElem& elem);

  // reads the remaining input
  std::vector<DatasetElem> readAll();
  void readAll(std::vector<DatasetElem>& dataset);

  // parses a whole text buffer (lines separated by '\n') on `nthreads` threads
  static void parseBuffer(const char* data, size_t size, std::vector<DatasetElem>& out,
                          size_t nthreads);

 private:
  std::string fileName_;
  std::unique_ptr<std::istream> stream_;
  std::string line_;
};

}  // namespace qmf
