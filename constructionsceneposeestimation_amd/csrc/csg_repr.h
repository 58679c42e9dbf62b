// csg_repr.h — Python's repr(float) for a finite double, in C++ (shared by
// the label-JSON encoders csg_json.cpp and csg_io.cpp): the shortest
// round-trip digits (std::to_chars, as Python's dtoa mode 0) laid out by
// repr's rules -- exponent form ("1e-05", "1.5e+16") when the decimal point
// lies more than 16 places right or 4 places left of the first digit, else
// fixed with at least one fractional digit ("3.0", "0.0001").
#pragma once
#include <charconv>
#include <cstdint>

namespace csg {

// Writes at most 32 bytes; returns the end.
inline char* repr_double(char* o, double x) {
  char sci[40];
  const auto r = std::to_chars(sci, sci + sizeof sci, x, std::chars_format::scientific);
  const char* p = sci;
  const char* end = r.ptr;
  if (*p == '-') {
    *o++ = '-';
    ++p;
  }
  char dig[24] = {0};
  int nd = 0;
  while (p < end && *p != 'e') {
    if (*p != '.') dig[nd++] = *p;
    ++p;
  }
  int e10 = 0;   // "e+XX" / "e-XX" (not NUL-terminated)
  std::from_chars(p + 1 + (p[1] == '+'), end, e10);
  const int decpt = e10 + 1;   // value = 0.d1d2... x 10^decpt
  if (decpt <= -4 || decpt > 16) {
    *o++ = dig[0];
    if (nd > 1) {
      *o++ = '.';
      for (int k = 1; k < nd; ++k) *o++ = dig[k];
    }
    *o++ = 'e';
    int ex = decpt - 1;
    *o++ = ex < 0 ? '-' : '+';
    if (ex < 0) ex = -ex;
    if (ex < 10) *o++ = '0';
    o = std::to_chars(o, o + 4, ex).ptr;
  } else if (decpt <= 0) {
    *o++ = '0';
    *o++ = '.';
    for (int k = 0; k < -decpt; ++k) *o++ = '0';
    for (int k = 0; k < nd; ++k) *o++ = dig[k];
  } else if (decpt >= nd) {
    for (int k = 0; k < nd; ++k) *o++ = dig[k];
    for (int k = nd; k < decpt; ++k) *o++ = '0';
    *o++ = '.';
    *o++ = '0';
  } else {
    for (int k = 0; k < decpt; ++k) *o++ = dig[k];
    *o++ = '.';
    for (int k = decpt; k < nd; ++k) *o++ = dig[k];
  }
  return o;
}

}  // namespace csg
