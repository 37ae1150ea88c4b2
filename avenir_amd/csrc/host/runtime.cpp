// Host runtime glue: HIP error reporting (turned into Python exceptions by pybind11).
#include <hip/hip_runtime.h>
#include <sstream>
#include <stdexcept>

void av_report_hip_error(hipError_t e, const char* expr, const char* file, int line) {
  std::ostringstream os;
  os << "HIP error " << static_cast<int>(e) << " (" << hipGetErrorString(e) << ") at " << file << ":"
     << line << " in `" << expr << "`";
  throw std::runtime_error(os.str());
}
