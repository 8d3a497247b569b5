// ato_dual.hpp -- forward-mode dual numbers for the templated model / segment programs.
//
// Dual<T, ND> carries a value and ND tangents. Instantiating a program with T = Dual
// differentiates it exactly (no truncation error) along ND seeded directions:
//   * the RK4 transcription differentiates the 4-stage integrator through the model's VALUE
//     path (the hand-derived Jacobian rows the model also produces are dead code there and
//     are dropped by the compiler),
//   * the Hessian of the Lagrangian differentiates the hand-derived Jacobians themselves
//     along coloured seed directions.
// Only the operations the programs use are provided.
#pragma once
#include "ato_models.hpp"

namespace ato {

template <class T, int ND>
struct Dual {
    T v;
    T d[ND];
    ATO_HD Dual() : v(T(0)) {
#pragma unroll
        for (int i = 0; i < ND; ++i) d[i] = T(0);
    }
    ATO_HD Dual(double x) : v(T(x)) {     // NOLINT: constants convert implicitly, as for T
#pragma unroll
        for (int i = 0; i < ND; ++i) d[i] = T(0);
    }
    ATO_HD Dual(float x) : v(T(x)) {      // NOLINT
#pragma unroll
        for (int i = 0; i < ND; ++i) d[i] = T(0);
    }
    ATO_HD Dual(int x) : v(T(x)) {        // NOLINT
#pragma unroll
        for (int i = 0; i < ND; ++i) d[i] = T(0);
    }
    ATO_HD static Dual seed(T x, int dir) {
        Dual r;
        r.v = x;
#pragma unroll
        for (int i = 0; i < ND; ++i) r.d[i] = T(i == dir ? 1 : 0);
        return r;
    }
    ATO_HD Dual& operator+=(const Dual& b) {
        v += b.v;
#pragma unroll
        for (int i = 0; i < ND; ++i) d[i] += b.d[i];
        return *this;
    }
    ATO_HD Dual& operator-=(const Dual& b) {
        v -= b.v;
#pragma unroll
        for (int i = 0; i < ND; ++i) d[i] -= b.d[i];
        return *this;
    }
    ATO_HD Dual& operator*=(const Dual& b) {
#pragma unroll
        for (int i = 0; i < ND; ++i) d[i] = d[i] * b.v + v * b.d[i];
        v *= b.v;
        return *this;
    }
};

template <class T, int ND>
ATO_HD Dual<T, ND> operator-(const Dual<T, ND>& a) {
    Dual<T, ND> r;
    r.v = -a.v;
#pragma unroll
    for (int i = 0; i < ND; ++i) r.d[i] = -a.d[i];
    return r;
}
template <class T, int ND>
ATO_HD Dual<T, ND> operator+(const Dual<T, ND>& a, const Dual<T, ND>& b) {
    Dual<T, ND> r = a;
    r += b;
    return r;
}
template <class T, int ND>
ATO_HD Dual<T, ND> operator-(const Dual<T, ND>& a, const Dual<T, ND>& b) {
    Dual<T, ND> r = a;
    r -= b;
    return r;
}
template <class T, int ND>
ATO_HD Dual<T, ND> operator*(const Dual<T, ND>& a, const Dual<T, ND>& b) {
    Dual<T, ND> r;
    r.v = a.v * b.v;
#pragma unroll
    for (int i = 0; i < ND; ++i) r.d[i] = a.d[i] * b.v + a.v * b.d[i];
    return r;
}
template <class T, int ND>
ATO_HD Dual<T, ND> operator/(const Dual<T, ND>& a, const Dual<T, ND>& b) {
    Dual<T, ND> r;
    const T ib = T(1) / b.v;
    r.v = a.v * ib;
#pragma unroll
    for (int i = 0; i < ND; ++i) r.d[i] = (a.d[i] - r.v * b.d[i]) * ib;
    return r;
}
// mixed with plain numbers (int / double literals and T constants)
template <class T, int ND>
ATO_HD Dual<T, ND> operator*(double a, const Dual<T, ND>& b) { return Dual<T, ND>(a) * b; }
template <class T, int ND>
ATO_HD Dual<T, ND> operator*(const Dual<T, ND>& a, double b) { return a * Dual<T, ND>(b); }
template <class T, int ND>
ATO_HD Dual<T, ND> operator+(double a, const Dual<T, ND>& b) { return Dual<T, ND>(a) + b; }
template <class T, int ND>
ATO_HD Dual<T, ND> operator+(const Dual<T, ND>& a, double b) { return a + Dual<T, ND>(b); }
template <class T, int ND>
ATO_HD Dual<T, ND> operator-(double a, const Dual<T, ND>& b) { return Dual<T, ND>(a) - b; }
template <class T, int ND>
ATO_HD Dual<T, ND> operator-(const Dual<T, ND>& a, double b) { return a - Dual<T, ND>(b); }
template <class T, int ND>
ATO_HD Dual<T, ND> operator/(double a, const Dual<T, ND>& b) { return Dual<T, ND>(a) / b; }
template <class T, int ND>
ATO_HD Dual<T, ND> operator/(const Dual<T, ND>& a, double b) { return a / Dual<T, ND>(b); }

template <class T, int ND>
ATO_HD Dual<T, ND> tsqrt(Dual<T, ND> a) {
    Dual<T, ND> r;
    r.v = tsqrt(a.v);
    const T h = T(0.5) / r.v;
#pragma unroll
    for (int i = 0; i < ND; ++i) r.d[i] = a.d[i] * h;
    return r;
}
template <class T, int ND>
ATO_HD Dual<T, ND> tsin(Dual<T, ND> a) {
    Dual<T, ND> r;
    r.v = tsin(a.v);
    const T c = tcos(a.v);
#pragma unroll
    for (int i = 0; i < ND; ++i) r.d[i] = a.d[i] * c;
    return r;
}
template <class T, int ND>
ATO_HD Dual<T, ND> tcos(Dual<T, ND> a) {
    Dual<T, ND> r;
    r.v = tcos(a.v);
    const T s = -tsin(a.v);
#pragma unroll
    for (int i = 0; i < ND; ++i) r.d[i] = a.d[i] * s;
    return r;
}

// value part of a plain number or a dual
template <class T>
ATO_HD T value_of(const T& x) { return x; }
template <class T, int ND>
ATO_HD T value_of(const Dual<T, ND>& x) { return x.v; }

}  // namespace ato
