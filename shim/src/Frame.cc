// Frame's static image bounds (src/Frame.cc:33-34 defines them for the reference).
#include "Frame.h"

namespace ORB_SLAM2 {
float Frame::mnMinX, Frame::mnMaxX, Frame::mnMinY, Frame::mnMaxY;
}
