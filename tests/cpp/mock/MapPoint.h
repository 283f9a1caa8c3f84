/* TEST-ONLY mock of the MapPoint accessors ORBmatcher reads (isBad). */
#ifndef MAPPOINT_H
#define MAPPOINT_H
namespace ORB_SLAM2 {
class MapPoint {
public:
    bool bad = false;
    bool isBad() { return bad; }
};
}  // namespace ORB_SLAM2
#endif
