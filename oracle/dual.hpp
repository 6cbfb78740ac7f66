// ORACLE — TEST INFRASTRUCTURE ONLY (see physics.hpp header).
//
// Forward-mode dual numbers: the oracle's physics is templated on its scalar type, so
// instantiating it with Dual<N> yields the exact Jacobian of the fp64 oracle step with respect to
// up to N seeded inputs. This is the derivative reference for the HIP step adjoint (APG, reference
// train_apg.py:161-209 differentiates through mjx.step): branches follow the primal values, so the
// result is the derivative of the branch the primal takes, as reverse-mode autodiff of MJX gives.
#pragma once
#include <cmath>

namespace oracle {

template <int N> struct Dual {
  double v;
  double d[N];
  Dual() : v(0) { for (int i = 0; i < N; i++) d[i] = 0; }
  Dual(double x) : v(x) { for (int i = 0; i < N; i++) d[i] = 0; }  // NOLINT: implicit on purpose
  explicit operator double() const { return v; }
  Dual& operator+=(const Dual& o) { v += o.v; for (int i = 0; i < N; i++) d[i] += o.d[i]; return *this; }
  Dual& operator-=(const Dual& o) { v -= o.v; for (int i = 0; i < N; i++) d[i] -= o.d[i]; return *this; }
  Dual& operator*=(const Dual& o) { *this = *this * o; return *this; }
  Dual& operator/=(const Dual& o) { *this = *this / o; return *this; }
  friend Dual operator-(const Dual& a) { Dual r; r.v = -a.v; for (int i = 0; i < N; i++) r.d[i] = -a.d[i]; return r; }
  friend Dual operator+(const Dual& a, const Dual& b) { Dual r = a; r += b; return r; }
  friend Dual operator-(const Dual& a, const Dual& b) { Dual r = a; r -= b; return r; }
  friend Dual operator*(const Dual& a, const Dual& b) {
    Dual r; r.v = a.v * b.v;
    for (int i = 0; i < N; i++) r.d[i] = a.d[i] * b.v + a.v * b.d[i];
    return r;
  }
  friend Dual operator/(const Dual& a, const Dual& b) {
    Dual r; r.v = a.v / b.v;
    const double ib = 1.0 / b.v;
    for (int i = 0; i < N; i++) r.d[i] = (a.d[i] - r.v * b.d[i]) * ib;
    return r;
  }
  friend bool operator<(const Dual& a, const Dual& b) { return a.v < b.v; }
  friend bool operator>(const Dual& a, const Dual& b) { return a.v > b.v; }
  friend bool operator<=(const Dual& a, const Dual& b) { return a.v <= b.v; }
  friend bool operator>=(const Dual& a, const Dual& b) { return a.v >= b.v; }
  friend bool operator==(const Dual& a, const Dual& b) { return a.v == b.v; }
  friend bool operator!=(const Dual& a, const Dual& b) { return a.v != b.v; }
  // chain rule helper: f(v) with derivative df
  Dual apply(double fv, double df) const { Dual r; r.v = fv; for (int i = 0; i < N; i++) r.d[i] = df * d[i]; return r; }
};

}  // namespace oracle

namespace std {
template <int N> oracle::Dual<N> sqrt(const oracle::Dual<N>& a) { double s = std::sqrt(a.v); return a.apply(s, s > 0 ? 0.5 / s : 0.0); }
template <int N> oracle::Dual<N> sin(const oracle::Dual<N>& a) { return a.apply(std::sin(a.v), std::cos(a.v)); }
template <int N> oracle::Dual<N> cos(const oracle::Dual<N>& a) { return a.apply(std::cos(a.v), -std::sin(a.v)); }
template <int N> oracle::Dual<N> abs(const oracle::Dual<N>& a) { return a.apply(std::abs(a.v), a.v < 0 ? -1.0 : 1.0); }
template <int N> oracle::Dual<N> asin(const oracle::Dual<N>& a) { return a.apply(std::asin(a.v), 1.0 / std::sqrt(1.0 - a.v * a.v)); }
template <int N> oracle::Dual<N> atan2(const oracle::Dual<N>& y, const oracle::Dual<N>& x) {
  oracle::Dual<N> r; r.v = std::atan2(y.v, x.v);
  const double den = x.v * x.v + y.v * y.v;
  for (int i = 0; i < N; i++) r.d[i] = (x.v * y.d[i] - y.v * x.d[i]) / den;
  return r;
}
template <int N> oracle::Dual<N> pow(const oracle::Dual<N>& a, const oracle::Dual<N>& b) {
  oracle::Dual<N> r; r.v = std::pow(a.v, b.v);
  const double da = a.v != 0 ? b.v * std::pow(a.v, b.v - 1) : 0.0, db = a.v > 0 ? r.v * std::log(a.v) : 0.0;
  for (int i = 0; i < N; i++) r.d[i] = da * a.d[i] + db * b.d[i];
  return r;
}
template <int N> bool isfinite(const oracle::Dual<N>& a) { return std::isfinite(a.v); }
}  // namespace std
