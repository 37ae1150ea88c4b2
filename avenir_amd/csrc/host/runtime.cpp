// Host runtime glue: HIP error reporting (turned into Python exceptions by pybind11).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <sstream>
#include <stdexcept>

void av_report_hip_error(hipError_t e, const char* expr, const char* file, int line) {
  std::ostringstream os;
  os << "HIP error " << static_cast<int>(e) << " (" << hipGetErrorString(e) << ") at " << file << ":"
     << line << " in `" << expr << "`";
  throw std::runtime_error(os.str());
}

namespace av {

int resident_blocks(const void* kernel, int block, size_t lds) {
  int dev = 0, cus = 0, per_cu = 0;
  hipError_t e;
  if ((e = hipGetDevice(&dev)) != hipSuccess) av_report_hip_error(e, "hipGetDevice", __FILE__, __LINE__);
  if ((e = hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev)) != hipSuccess)
    av_report_hip_error(e, "hipDeviceGetAttribute", __FILE__, __LINE__);
  if ((e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kernel, block, lds)) != hipSuccess)
    av_report_hip_error(e, "hipOccupancyMaxActiveBlocksPerMultiprocessor", __FILE__, __LINE__);
  return std::max(1, per_cu) * std::max(1, cus);
}

}  // namespace av
