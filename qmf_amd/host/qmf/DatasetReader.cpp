#include <qmf/DatasetReader.h>

#include <cctype>
#include <charconv>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <sstream>

#include <qmf/utils/Log.h>
#include <qmf/utils/ParallelExecutor.h>

namespace qmf {

namespace {

[[noreturn]] void badLine(const char* b, const char* e) {
  LOG(FATAL) << "Check failed: result == 3 the file format is incorrect: " << std::string(b, e);
  std::abort();
}

// "%lld %lld %lf" on [b, e) (e points at the line terminator, not included).  Returns
// false when fewer than three conversions succeed, like sscanf's result != 3.  The buffer
// is copied into a small NUL-terminated scratch so strtoll/strtod cannot run past the line.
bool parseLineCopy(const char* b, const char* e, DatasetElem& elem, std::string& scratch) {
  scratch.assign(b, e);
  const char* p = scratch.c_str();
  char* q = nullptr;
  errno = 0;
  const long long u = std::strtoll(p, &q, 10);
  if (q == p) return false;
  p = q;
  const long long i = std::strtoll(p, &q, 10);
  if (q == p) return false;
  p = q;
  const double v = std::strtod(p, &q);
  if (q == p) return false;
  elem.userId = u;
  elem.itemId = i;
  elem.value = static_cast<Double>(v);
  return true;
}

inline bool isSpace(char c) { return c == ' ' || (c >= '\t' && c <= '\r'); }

// The same conversion in place, without the copy: std::from_chars reads [b, e) directly and
// rounds like strtod / strtoll on plain decimal fields.  Anything it does not take the way
// sscanf would (a '+' sign, hex or inf/nan values, overflow, a field it rejects) goes to
// parseLineCopy, so the result is sscanf's in every case.
bool parseLine(const char* b, const char* e, DatasetElem& elem, std::string& scratch) {
  const char* p = b;
  long long f[2];
  for (int j = 0; j < 2; ++j) {
    while (p < e && isSpace(*p)) ++p;
    const auto r = std::from_chars(p, e, f[j]);
    if (r.ec != std::errc() || (r.ptr < e && !isSpace(*r.ptr)))
      return parseLineCopy(b, e, elem, scratch);
    p = r.ptr;
  }
  while (p < e && isSpace(*p)) ++p;
  double v = 0.0;
  const auto r = std::from_chars(p, e, v, std::chars_format::general);
  // a value field must end the number the way strtod would (whitespace, end of line, or a
  // character strtod also stops at); hex / inf / nan / '+' forms and range errors take the
  // exact path
  if (r.ec != std::errc() || r.ptr == p || (r.ptr < e && (isalnum((unsigned char)*r.ptr) ||
                                                          *r.ptr == '.' || *r.ptr == 'x')))
    return parseLineCopy(b, e, elem, scratch);
  elem.userId = f[0];
  elem.itemId = f[1];
  elem.value = static_cast<Double>(v);
  return true;
}

}  // namespace

DatasetReader::DatasetReader(const std::string& fileName) : fileName_(fileName) {}

DatasetReader::DatasetReader(std::unique_ptr<std::istream> stream) : stream_(std::move(stream)) {}

bool DatasetReader::readOne(DatasetElem& elem) {
  if (!stream_ && !fileName_.empty()) stream_ = std::make_unique<std::ifstream>(fileName_);
  CHECK(stream_);
  if (!std::getline(*stream_, line_)) return false;
  double value = 0.0;
  long long u = 0, i = 0;
  const int result = sscanf(line_.c_str(), "%lld %lld %lf", &u, &i, &value);
  CHECK_EQ(result, 3) << "the file format is incorrect: " << line_;
  elem.userId = u;
  elem.itemId = i;
  elem.value = static_cast<Double>(value);
  return true;
}

void DatasetReader::parseBuffer(const char* data, size_t size, std::vector<DatasetElem>& out,
                                size_t nthreads) {
  out.clear();
  if (size == 0) return;
  // chunk boundaries at line starts
  const size_t nt = std::max<size_t>(1, std::min(nthreads, size / (1 << 20) + 1));
  std::vector<size_t> start(nt + 1, size);
  start[0] = 0;
  for (size_t t = 1; t < nt; ++t) {
    size_t p = size * t / nt;
    if (p < start[t - 1]) p = start[t - 1];
    while (p < size && data[p - 1] != '\n') ++p;
    start[t] = p;
  }
  std::vector<std::vector<DatasetElem>> parts(nt);
  std::vector<size_t> badAt(nt, SIZE_MAX);
  ParallelExecutor::run(nt, [&](const size_t t) {
    std::string scratch;
    auto& v = parts[t];
    v.reserve((start[t + 1] - start[t]) / 12 + 1);
    size_t p = start[t];
    const size_t end = start[t + 1];
    while (p < end) {
      const char* nl = static_cast<const char*>(memchr(data + p, '\n', end - p));
      const size_t le = nl ? static_cast<size_t>(nl - data) : end;
      DatasetElem elem;
      if (!parseLine(data + p, data + le, elem, scratch)) {
        badAt[t] = p;
        return;
      }
      v.push_back(elem);
      p = le + 1;
    }
  });
  for (size_t t = 0; t < nt; ++t)
    if (badAt[t] != SIZE_MAX) {
      const char* b = data + badAt[t];
      const char* nl = static_cast<const char*>(memchr(b, '\n', size - badAt[t]));
      badLine(b, nl ? nl : data + size);
    }
  size_t total = 0;
  for (const auto& v : parts) total += v.size();
  out.reserve(total);
  for (auto& v : parts) {
    out.insert(out.end(), v.begin(), v.end());
    std::vector<DatasetElem>().swap(v);
  }
}

void DatasetReader::readAll(std::vector<DatasetElem>& dataset) {
  dataset.clear();
  if (!stream_ && !fileName_.empty()) {
    // whole-file fast path
    FILE* f = std::fopen(fileName_.c_str(), "rb");
    if (!f) return;  // the reference's ifstream on a missing file reads nothing
    std::string buf;
    std::fseek(f, 0, SEEK_END);
    const long sz = std::ftell(f);
    std::fseek(f, 0, SEEK_SET);
    if (sz > 0) {
      buf.resize(static_cast<size_t>(sz));
      const size_t got = std::fread(&buf[0], 1, buf.size(), f);
      buf.resize(got);
    }
    std::fclose(f);
    fileName_.clear();
    stream_ = std::make_unique<std::istringstream>(std::string());  // consumed
    const unsigned hc = std::thread::hardware_concurrency();
    parseBuffer(buf.data(), buf.size(), dataset, std::min<unsigned>(hc ? hc : 1, 32));
    return;
  }
  DatasetElem elem;
  while (readOne(elem)) dataset.push_back(elem);
}

std::vector<DatasetElem> DatasetReader::readAll() {
  std::vector<DatasetElem> dataset;
  readAll(dataset);
  return dataset;
}

}  // namespace qmf
