// Minimal OpenCV 3.x core surface for compiling the liborbx shim without
// OpenCV: only the members ORBextractor.cc / ORBmatcher.cc / Frame touch
// (cv::Mat of CV_8U or CV_32F elements, cv::KeyPoint, cv::Point2f,
// InputArray/OutputArray).
// Layouts follow OpenCV where the shim relies on them: cv::KeyPoint is
// pt.x, pt.y, size, angle, response, octave, class_id (28 bytes) and
// cv::Point2f is two floats. Not a general OpenCV replacement.
#ifndef ORBX_CV_STUB_CORE_HPP
#define ORBX_CV_STUB_CORE_HPP

#include <cassert>
#include <cstddef>
#include <cstring>
#include <memory>
#include <vector>

#define CV_8U 0
#define CV_8UC1 0
#define CV_32F 5

typedef unsigned char uchar;

namespace cv {

class _OutputArray;

struct Point2f {
  float x = 0.f, y = 0.f;
  Point2f() = default;
  Point2f(float x_, float y_) : x(x_), y(y_) {}
};

struct Point2i {
  int x = 0, y = 0;
  Point2i() = default;
  Point2i(int x_, int y_) : x(x_), y(y_) {}
};
typedef Point2i Point;

struct KeyPoint {
  Point2f pt;
  float size = 0.f, angle = -1.f, response = 0.f;
  int octave = 0, class_id = -1;
  KeyPoint() = default;
  KeyPoint(Point2f p, float s, float a = -1.f, float r = 0.f, int o = 0, int c = -1)
      : pt(p), size(s), angle(a), response(r), octave(o), class_id(c) {}
};

// Single-channel matrix of CV_8U or CV_32F elements with row stride `step`
// (bytes); owns its buffer unless it wraps external data (Mat(rows, cols,
// type, data, step)) or is a row / column view.
class Mat {
 public:
  int rows = 0, cols = 0;
  size_t step = 0;
  uchar* data = nullptr;

  Mat() = default;
  Mat(int r, int c, int type) { create(r, c, type); }
  Mat(int r, int c, int type, void* ext, size_t stp = 0)
      : rows(r), cols(c), step(stp ? stp : (size_t)c * esize(type)), data((uchar*)ext), type_(type) {}

  static size_t esize(int type) {
    assert(type == CV_8U || type == CV_32F);
    return type == CV_32F ? 4 : 1;
  }
  void create(int r, int c, int type) {
    if (buf_ && rows == r && cols == c && type_ == type && step == (size_t)c * esize(type)) return;
    buf_ = std::make_shared<std::vector<uchar>>((size_t)r * c * esize(type));
    rows = r;
    cols = c;
    type_ = type;
    step = (size_t)c * esize(type);
    data = buf_->data();
  }
  void release() { *this = Mat(); }
  bool empty() const { return data == nullptr || rows == 0 || cols == 0; }
  int type() const { return type_; }
  int channels() const { return 1; }
  size_t elemSize() const { return esize(type_); }
  bool isContinuous() const { return step == (size_t)cols * elemSize() || rows == 1; }

  Mat row(int i) const { return rowRange(i, i + 1); }
  Mat col(int j) const { return colRange(j, j + 1); }
  Mat rowRange(int a, int b) const {
    Mat m(*this);
    m.rows = b - a;
    m.data = data + (size_t)a * step;
    return m;
  }
  Mat colRange(int a, int b) const {
    Mat m(*this);
    m.cols = b - a;
    m.data = data + (size_t)a * elemSize();
    return m;
  }
  Mat clone() const {
    Mat m(rows, cols, type_);
    for (int r = 0; r < rows; ++r) memcpy(m.data + (size_t)r * m.step, data + (size_t)r * step, cols * elemSize());
    return m;
  }
  void copyTo(Mat& dst) const {
    dst.create(rows, cols, type_);
    for (int r = 0; r < rows; ++r) memcpy(dst.data + (size_t)r * dst.step, data + (size_t)r * step, cols * elemSize());
  }
  void copyTo(const _OutputArray& dst) const;
  template <typename T> T* ptr(int r = 0) { return (T*)(data + (size_t)r * step); }
  template <typename T> const T* ptr(int r = 0) const { return (const T*)(data + (size_t)r * step); }
  template <typename T> T& at(int r, int c) { return ptr<T>(r)[c]; }
  template <typename T> const T& at(int r, int c) const { return ptr<T>(r)[c]; }
  // element i of a row or column vector
  template <typename T> T& at(int i) { return rows == 1 ? at<T>(0, i) : at<T>(i, 0); }
  template <typename T> const T& at(int i) const { return rows == 1 ? at<T>(0, i) : at<T>(i, 0); }

 private:
  std::shared_ptr<std::vector<uchar>> buf_;
  int type_ = CV_8U;
};

class _InputArray {
 public:
  _InputArray() = default;
  _InputArray(const Mat& m) : m_(&m) {}
  Mat getMat() const { return m_ ? *m_ : Mat(); }
  bool empty() const { return !m_ || m_->empty(); }

 private:
  const Mat* m_ = nullptr;
};

class _OutputArray {
 public:
  _OutputArray(Mat& m) : m_(&m) {}
  void create(int r, int c, int type) const { m_->create(r, c, type); }
  void release() const { m_->release(); }
  Mat& getMatRef() const { return *m_; }
  Mat getMat() const { return *m_; }

 private:
  Mat* m_;
};

typedef const _InputArray& InputArray;
typedef const _OutputArray& OutputArray;

inline void Mat::copyTo(const _OutputArray& dst) const { copyTo(dst.getMatRef()); }

inline const _InputArray& noArray() {
  static _InputArray none;
  return none;
}

}  // namespace cv

#endif
