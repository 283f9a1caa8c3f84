/* TEST-ONLY minimal stand-in for the few OpenCV types the drop-in classes
 * (cooperative-orb-slam_amd/host/) use, so they compile and run in this OpenCV-less image.
 * It is never used to build reference code. Real deployments compile against OpenCV. */
#ifndef CVMIN_CORE_HPP
#define CVMIN_CORE_HPP
#include <cstddef>
#include <cstring>
#include <memory>
#include <vector>

#define CV_8U 0
#define CV_8UC1 0
#define CV_32F 5

namespace cv {
struct Point2f { float x = 0, y = 0; Point2f() {} Point2f(float a, float b) : x(a), y(b) {} };
class Mat {
public:
    int rows = 0, cols = 0, tp = CV_8U;
    size_t step = 0;
    unsigned char* data = nullptr;
    std::shared_ptr<std::vector<unsigned char> > store;
    Mat() {}
    Mat(int r, int c, int t) { create(r, c, t); }
    Mat(int r, int c, int t, void* d, size_t st = 0) : rows(r), cols(c), tp(t), step(st ? st : c * esz(t)), data((unsigned char*)d) {}
    static size_t esz(int t) { return t == CV_32F ? 4 : 1; }
    void create(int r, int c, int t) {
        if (data && rows == r && cols == c && tp == t) return;
        rows = r; cols = c; tp = t; step = (size_t)c * esz(t);
        store = std::make_shared<std::vector<unsigned char> >(step * r);
        data = store->data();
    }
    void release() { rows = cols = 0; step = 0; data = nullptr; store.reset(); }
    bool empty() const { return data == nullptr || rows == 0 || cols == 0; }
    int type() const { return tp; }
    bool isContinuous() const { return step == (size_t)cols * esz(tp) || rows <= 1; }
    Mat clone() const {
        Mat m(rows, cols, tp);
        for (int i = 0; i < rows; i++) memcpy(m.data + i * m.step, data + i * step, m.step);
        return m;
    }
    Mat row(int i) const { Mat m(*this); m.rows = 1; m.data = data + i * step; return m; }
    template <class T> T* ptr(int i = 0) { return (T*)(data + i * step); }
    template <class T> const T* ptr(int i = 0) const { return (const T*)(data + i * step); }
    template <class T> T& at(int i, int j) { return ((T*)(data + i * step))[j]; }
    template <class T> const T& at(int i, int j) const { return ((const T*)(data + i * step))[j]; }
    template <class T> T& at(int i) { return ((T*)data)[i]; }
};
class _InputArray {
public:
    const Mat* m;
    _InputArray(const Mat& x) : m(&x) {}
    Mat getMat() const { return *m; }
    bool empty() const { return m->empty(); }
};
class _OutputArray {
public:
    Mat* m;
    _OutputArray(Mat& x) : m(&x) {}
    void create(int r, int c, int t) const { m->create(r, c, t); }
    void release() const { m->release(); }
    Mat getMat() const { return *m; }
};
typedef const _InputArray& InputArray;
typedef const _OutputArray& OutputArray;
inline Mat noArray() { return Mat(); }
}  // namespace cv
#endif
