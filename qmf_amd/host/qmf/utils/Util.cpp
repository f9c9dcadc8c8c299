#include <qmf/utils/Util.h>

namespace qmf {

std::vector<std::string> split(const std::string& str, const char delim) {
  std::vector<std::string> out;
  if (str.empty()) return out;
  size_t start = 0;
  for (;;) {
    const size_t end = str.find(delim, start);
    out.emplace_back(str, start, end == std::string::npos ? std::string::npos : end - start);
    if (end == std::string::npos) break;
    start = end + 1;
  }
  return out;
}

}  // namespace qmf
