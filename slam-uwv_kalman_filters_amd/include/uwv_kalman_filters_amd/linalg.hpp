// linalg.hpp — the value types of the facade's single-filter (reference) call forms.
//
// The reference passes Eigen fixed-size types everywhere (PoseUKF.hpp:100-190:
// Eigen::Vector3d, Matrix3d, Quaterniond, Affine3d, the MEASUREMENT types' Mu /
// Cov, PoseUKFConfig.hpp's base::Vector3d / Vector6d / VectorXd).  Where Eigen
// is installed these names ARE Eigen's (a caller's Eigen objects bind directly);
// where it is not (this build image), the small column-major types below stand
// in with the subset of Eigen's interface those call sites use: element access
// (i, j) / (i) / [i] / x() y() z(), Zero / Identity / Ones / Constant / UnitX..Z,
// the comma initializer (row-major fill order, as Eigen's), + - * and
// transpose, Quaterniond (w, x, y, z) with AngleAxisd and rotation-matrix
// conversions, and Affine3d's translation() / linear() / rotation().
// Define UWVK_FACADE_NO_EIGEN to use these types even when Eigen is present.
#pragma once
#include <array>
#include <cmath>
#include <cstddef>
#include <stdexcept>
#include <type_traits>
#include <vector>

#if !defined(UWVK_FACADE_NO_EIGEN) && __has_include(<Eigen/Core>) && __has_include(<Eigen/Geometry>)
#include <Eigen/Core>
#include <Eigen/Geometry>
#define UWVK_FACADE_EIGEN 1
namespace uwv_kalman_filters_amd {
template <int R, int C>
using Matrix = Eigen::Matrix<double, R, C>;
using VectorXd = Eigen::VectorXd;
using Quaterniond = Eigen::Quaterniond;
using AngleAxisd = Eigen::AngleAxisd;
using Affine3d = Eigen::Affine3d;
}  // namespace uwv_kalman_filters_amd
#else
#define UWVK_FACADE_EIGEN 0
namespace uwv_kalman_filters_amd {

// Fixed-size R x C matrix of doubles, column-major like Eigen's default.
template <int R, int C>
class Matrix {
  static_assert(R > 0 && C > 0, "fixed sizes only");

 public:
  static constexpr int RowsAtCompileTime = R, ColsAtCompileTime = C, SizeAtCompileTime = R * C;
  Matrix() : a_{} {}
  // Vector2d(x, y), Vector3d(x, y, z), Vector4d(x, y, z, w): Eigen's vector constructors
  template <class... T, class = std::enable_if_t<C == 1 && (R >= 2 && R <= 4) && sizeof...(T) == R &&
                                                 (std::is_arithmetic<T>::value && ...)>>
  Matrix(T... v) : a_{{static_cast<double>(v)...}} {}

  static constexpr int rows() { return R; }
  static constexpr int cols() { return C; }
  static constexpr int size() { return R * C; }
  double& operator()(int i, int j) { return a_[(size_t)j * R + i]; }
  double operator()(int i, int j) const { return a_[(size_t)j * R + i]; }
  double& operator()(int i) { return a_[i]; }  // linear (column-major) index, as Eigen's
  double operator()(int i) const { return a_[i]; }
  double& operator[](int i) { return a_[i]; }
  double operator[](int i) const { return a_[i]; }
  double& x() { return a_[0]; }
  double& y() { return a_[1]; }
  double& z() { return a_[2]; }
  double& w() { return a_[3]; }
  double x() const { return a_[0]; }
  double y() const { return a_[1]; }
  double z() const { return a_[2]; }
  double w() const { return a_[3]; }
  double* data() { return a_.data(); }
  const double* data() const { return a_.data(); }

  static Matrix Zero() { return Matrix(); }
  static Matrix Constant(double v) {
    Matrix m;
    m.a_.fill(v);
    return m;
  }
  static Matrix Ones() { return Constant(1.0); }
  static Matrix Identity() {
    Matrix m;
    for (int i = 0; i < (R < C ? R : C); i++) m(i, i) = 1.0;
    return m;
  }
  static Matrix Unit(int i) {
    Matrix m;
    m.a_[i] = 1.0;
    return m;
  }
  static Matrix UnitX() { return Unit(0); }
  static Matrix UnitY() { return Unit(1); }
  static Matrix UnitZ() { return Unit(2); }
  Matrix& setZero() { return *this = Zero(); }
  Matrix& setIdentity() { return *this = Identity(); }
  Matrix& setConstant(double v) { return *this = Constant(v); }

  Matrix<C, R> transpose() const {
    Matrix<C, R> t;
    for (int i = 0; i < R; i++)
      for (int j = 0; j < C; j++) t(j, i) = (*this)(i, j);
    return t;
  }
  Matrix operator-() const { return *this * -1.0; }
  Matrix operator+(const Matrix& o) const {
    Matrix r = *this;
    return r += o;
  }
  Matrix operator-(const Matrix& o) const {
    Matrix r = *this;
    return r -= o;
  }
  Matrix operator*(double s) const {
    Matrix r = *this;
    return r *= s;
  }
  Matrix operator/(double s) const { return *this * (1.0 / s); }
  friend Matrix operator*(double s, const Matrix& m) { return m * s; }
  Matrix& operator+=(const Matrix& o) {
    for (int k = 0; k < R * C; k++) a_[k] += o.a_[k];
    return *this;
  }
  Matrix& operator-=(const Matrix& o) {
    for (int k = 0; k < R * C; k++) a_[k] -= o.a_[k];
    return *this;
  }
  Matrix& operator*=(double s) {
    for (double& v : a_) v *= s;
    return *this;
  }
  template <int K>
  Matrix<R, K> operator*(const Matrix<C, K>& o) const {
    Matrix<R, K> r;
    for (int j = 0; j < K; j++)
      for (int k = 0; k < C; k++)
        for (int i = 0; i < R; i++) r(i, j) += (*this)(i, k) * o(k, j);
    return r;
  }
  bool operator==(const Matrix& o) const { return a_ == o.a_; }
  bool operator!=(const Matrix& o) const { return a_ != o.a_; }
  double squaredNorm() const {
    double s = 0;
    for (double v : a_) s += v * v;
    return s;
  }
  double norm() const { return std::sqrt(squaredNorm()); }
  double dot(const Matrix& o) const {
    double s = 0;
    for (int k = 0; k < R * C; k++) s += a_[k] * o.a_[k];
    return s;
  }
  Matrix normalized() const { return *this / norm(); }
  template <int RR = R, int CC = C, class = std::enable_if_t<RR == 3 && CC == 1>>
  Matrix cross(const Matrix& o) const {
    return Matrix(y() * o.z() - z() * o.y(), z() * o.x() - x() * o.z(), x() * o.y() - y() * o.x());
  }
  // v.asDiagonal() as a dense matrix (vectors)
  template <int CC = C, class = std::enable_if_t<CC == 1>>
  Matrix<R, R> asDiagonal() const {
    Matrix<R, R> d;
    for (int i = 0; i < R; i++) d(i, i) = a_[i];
    return d;
  }
  bool allFinite() const {
    for (double v : a_)
      if (!std::isfinite(v)) return false;
    return true;
  }

  // m << a, b, c, ...: row-major fill order, as Eigen's comma initializer
  class CommaInit {
   public:
    CommaInit(Matrix& m, double v) : m_(m) { put(v); }
    CommaInit& operator,(double v) {
      put(v);
      return *this;
    }
    ~CommaInit() noexcept(false) {
      if (k_ != R * C && !std::uncaught_exceptions())
        throw std::invalid_argument("comma initializer: wrong number of coefficients");
    }

   private:
    void put(double v) {
      if (k_ >= R * C) throw std::invalid_argument("comma initializer: too many coefficients");
      m_(k_ / C, k_ % C) = v;
      k_++;
    }
    Matrix& m_;
    int k_ = 0;
  };
  CommaInit operator<<(double v) { return CommaInit(*this, v); }

 private:
  std::array<double, (size_t)R * C> a_;
};

// Dynamic-size column vector (base::VectorXd of PoseUKFConfig.hpp:75-87).
class VectorXd {
 public:
  VectorXd() = default;
  explicit VectorXd(int n) : v_((size_t)n, 0.0) {}
  template <int R>
  VectorXd(const Matrix<R, 1>& m) : v_(m.data(), m.data() + R) {}
  int size() const { return (int)v_.size(); }
  int rows() const { return size(); }
  void resize(int n) { v_.resize((size_t)n); }
  double& operator()(int i) { return v_.at((size_t)i); }
  double operator()(int i) const { return v_.at((size_t)i); }
  double& operator[](int i) { return v_.at((size_t)i); }
  double operator[](int i) const { return v_.at((size_t)i); }
  double* data() { return v_.data(); }
  const double* data() const { return v_.data(); }
  static VectorXd Zero(int n) { return VectorXd(n); }
  static VectorXd Constant(int n, double c) {
    VectorXd r(n);
    for (double& x : r.v_) x = c;
    return r;
  }
  static VectorXd Ones(int n) { return Constant(n, 1.0); }
  VectorXd& setZero() {
    for (double& x : v_) x = 0.0;
    return *this;
  }

 private:
  std::vector<double> v_;
};

using Matrix3 = Matrix<3, 3>;
using Vector3 = Matrix<3, 1>;

class AngleAxisd;

// Unit quaternion, constructed (w, x, y, z) as Eigen's; coeffs() is (x, y, z, w).
class Quaterniond {
 public:
  Quaterniond() : w_(1), x_(0), y_(0), z_(0) {}
  Quaterniond(double w, double x, double y, double z) : w_(w), x_(x), y_(y), z_(z) {}
  inline explicit Quaterniond(const AngleAxisd& aa);
  // from a rotation matrix (Shepperd's method, as Eigen's)
  explicit Quaterniond(const Matrix3& R) {
    const double t = R(0, 0) + R(1, 1) + R(2, 2);
    if (t > 0) {
      double s = std::sqrt(t + 1.0);
      w_ = 0.5 * s;
      s = 0.5 / s;
      x_ = (R(2, 1) - R(1, 2)) * s;
      y_ = (R(0, 2) - R(2, 0)) * s;
      z_ = (R(1, 0) - R(0, 1)) * s;
    } else {
      int i = 0;
      if (R(1, 1) > R(0, 0)) i = 1;
      if (R(2, 2) > R(i, i)) i = 2;
      const int j = (i + 1) % 3, k = (j + 1) % 3;
      double s = std::sqrt(R(i, i) - R(j, j) - R(k, k) + 1.0);
      double v[3];
      v[i] = 0.5 * s;
      s = 0.5 / s;
      w_ = (R(k, j) - R(j, k)) * s;
      v[j] = (R(j, i) + R(i, j)) * s;
      v[k] = (R(k, i) + R(i, k)) * s;
      x_ = v[0];
      y_ = v[1];
      z_ = v[2];
    }
  }
  static Quaterniond Identity() { return Quaterniond(); }
  double& w() { return w_; }
  double& x() { return x_; }
  double& y() { return y_; }
  double& z() { return z_; }
  double w() const { return w_; }
  double x() const { return x_; }
  double y() const { return y_; }
  double z() const { return z_; }
  Matrix<4, 1> coeffs() const { return Matrix<4, 1>(x_, y_, z_, w_); }
  Vector3 vec() const { return Vector3(x_, y_, z_); }
  double squaredNorm() const { return w_ * w_ + x_ * x_ + y_ * y_ + z_ * z_; }
  double norm() const { return std::sqrt(squaredNorm()); }
  void normalize() { *this = normalized(); }
  Quaterniond normalized() const {
    const double n = norm();
    return Quaterniond(w_ / n, x_ / n, y_ / n, z_ / n);
  }
  Quaterniond conjugate() const { return Quaterniond(w_, -x_, -y_, -z_); }
  Quaterniond inverse() const {
    const double n2 = squaredNorm();
    return Quaterniond(w_ / n2, -x_ / n2, -y_ / n2, -z_ / n2);
  }
  Quaterniond operator*(const Quaterniond& b) const {
    return Quaterniond(w_ * b.w_ - x_ * b.x_ - y_ * b.y_ - z_ * b.z_, w_ * b.x_ + x_ * b.w_ + y_ * b.z_ - z_ * b.y_,
                       w_ * b.y_ - x_ * b.z_ + y_ * b.w_ + z_ * b.x_, w_ * b.z_ + x_ * b.y_ - y_ * b.x_ + z_ * b.w_);
  }
  Matrix3 toRotationMatrix() const {
    Matrix3 R;
    const double w = w_, x = x_, y = y_, z = z_;
    R(0, 0) = 1 - 2 * (y * y + z * z); R(0, 1) = 2 * (x * y - w * z);     R(0, 2) = 2 * (x * z + w * y);
    R(1, 0) = 2 * (x * y + w * z);     R(1, 1) = 1 - 2 * (x * x + z * z); R(1, 2) = 2 * (y * z - w * x);
    R(2, 0) = 2 * (x * z - w * y);     R(2, 1) = 2 * (y * z + w * x);     R(2, 2) = 1 - 2 * (x * x + y * y);
    return R;
  }
  Vector3 operator*(const Vector3& v) const { return toRotationMatrix() * v; }

 private:
  double w_, x_, y_, z_;
};

class AngleAxisd {
 public:
  AngleAxisd(double angle, const Vector3& axis) : angle_(angle), axis_(axis) {}
  explicit AngleAxisd(const Quaterniond& q) {
    const Vector3 v = q.vec();
    const double n = v.norm();
    angle_ = 2.0 * std::atan2(n, q.w());
    axis_ = n > 0 ? v / n : Vector3::UnitX();
  }
  double angle() const { return angle_; }
  const Vector3& axis() const { return axis_; }
  Matrix3 toRotationMatrix() const { return Quaterniond(*this).toRotationMatrix(); }
  Quaterniond operator*(const AngleAxisd& o) const { return Quaterniond(*this) * Quaterniond(o); }
  friend Quaterniond operator*(const Quaterniond& q, const AngleAxisd& a) { return q * Quaterniond(a); }
  friend Quaterniond operator*(const AngleAxisd& a, const Quaterniond& q) { return Quaterniond(a) * q; }

 private:
  double angle_;
  Vector3 axis_;
};

inline Quaterniond::Quaterniond(const AngleAxisd& aa) {
  const double h = 0.5 * aa.angle(), s = std::sin(h);
  w_ = std::cos(h);
  x_ = aa.axis().x() * s;
  y_ = aa.axis().y() * s;
  z_ = aa.axis().z() * s;
}

// Rigid transform (Eigen::Affine3d restricted to rotation + translation).
class Affine3d {
 public:
  Affine3d() : L_(Matrix3::Identity()) {}
  explicit Affine3d(const Quaterniond& q) : L_(q.toRotationMatrix()) {}
  explicit Affine3d(const AngleAxisd& a) : L_(a.toRotationMatrix()) {}
  static Affine3d Identity() { return Affine3d(); }
  Vector3& translation() { return t_; }
  const Vector3& translation() const { return t_; }
  Matrix3& linear() { return L_; }
  const Matrix3& linear() const { return L_; }
  Matrix3 rotation() const { return L_; }
  Affine3d& setIdentity() { return *this = Affine3d(); }
  Affine3d& translate(const Vector3& v) {
    t_ += L_ * v;
    return *this;
  }
  Affine3d& pretranslate(const Vector3& v) {
    t_ += v;
    return *this;
  }
  Affine3d& rotate(const Quaterniond& q) {
    L_ = L_ * q.toRotationMatrix();
    return *this;
  }
  Affine3d& prerotate(const Quaterniond& q) {
    const Matrix3 R = q.toRotationMatrix();
    L_ = R * L_;
    t_ = R * t_;
    return *this;
  }
  Affine3d operator*(const Affine3d& o) const {
    Affine3d r;
    r.L_ = L_ * o.L_;
    r.t_ = L_ * o.t_ + t_;
    return r;
  }
  Vector3 operator*(const Vector3& v) const { return L_ * v + t_; }
  Affine3d inverse() const {
    Affine3d r;
    r.L_ = L_.transpose();
    r.t_ = -(r.L_ * t_);
    return r;
  }

 private:
  Matrix3 L_;
  Vector3 t_;
};

}  // namespace uwv_kalman_filters_amd
#endif

namespace uwv_kalman_filters_amd {
using Vector2d = Matrix<2, 1>;
using Vector3d = Matrix<3, 1>;
using Vector4d = Matrix<4, 1>;
using Vector6d = Matrix<6, 1>;
using Matrix2d = Matrix<2, 2>;
using Matrix3d = Matrix<3, 3>;
using Matrix6d = Matrix<6, 6>;

namespace detail {
// row-major copy of any fixed-size matrix into the C ABI's layout
template <class M>
void put_rowmajor(const M& m, double* out) {
  for (int i = 0; i < (int)m.rows(); i++)
    for (int j = 0; j < (int)m.cols(); j++) out[(size_t)i * m.cols() + j] = m(i, j);
}
template <class M>
void get_rowmajor(const double* in, M& m) {
  for (int i = 0; i < (int)m.rows(); i++)
    for (int j = 0; j < (int)m.cols(); j++) m(i, j) = in[(size_t)i * m.cols() + j];
}
// {tx, ty, tz, qw, qx, qy, qz} of a rigid transform
inline void pose7_of(const Affine3d& a, double out[7]) {
  const Quaterniond q(Matrix3d(a.rotation()));
  for (int k = 0; k < 3; k++) out[k] = a.translation()(k);
  out[3] = q.w(); out[4] = q.x(); out[5] = q.y(); out[6] = q.z();
}
}  // namespace detail
}  // namespace uwv_kalman_filters_amd
