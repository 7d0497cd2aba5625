// cv::KeyPoint lives in the core stub.
#include "../core/core.hpp"
