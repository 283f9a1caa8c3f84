/* TEST-ONLY minimal stand-in (see core.hpp): cv::KeyPoint */
#ifndef CVMIN_FEATURES2D_HPP
#define CVMIN_FEATURES2D_HPP
#include "../core/core.hpp"
namespace cv {
class KeyPoint {
public:
    Point2f pt;
    float size = 0, angle = -1, response = 0;
    int octave = 0, class_id = -1;
    KeyPoint() {}
    KeyPoint(float x, float y, float sz, float a = -1, float r = 0, int o = 0, int c = -1)
        : pt(x, y), size(sz), angle(a), response(r), octave(o), class_id(c) {}
};
}  // namespace cv
#endif
