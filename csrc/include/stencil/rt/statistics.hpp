#pragma once
// Sample statistics for benchmark apps.
// Parity: reference bin/statistics.{hpp,cpp} (insert/avg/min/max/count/trimean/med/stddev).
// trimean = (Q1 + 2*Q2 + Q3)/4 with quartile index n/4*k as in statistics.cpp:25-34.
// Fix: med() of an even count is the mean of the two middle samples (the reference adds them, :36-46).
#include <algorithm>
#include <cmath>
#include <limits>
#include <vector>

class Statistics {
  std::vector<double> x_;

public:
  void insert(double v) { x_.push_back(v); }
  size_t count() const { return x_.size(); }
  double avg() const {
    if (x_.empty()) return std::numeric_limits<double>::quiet_NaN();
    double s = 0;
    for (double v : x_) s += v;
    return s / double(x_.size());
  }
  double min() const { return x_.empty() ? std::numeric_limits<double>::quiet_NaN() : *std::min_element(x_.begin(), x_.end()); }
  double max() const { return x_.empty() ? std::numeric_limits<double>::quiet_NaN() : *std::max_element(x_.begin(), x_.end()); }
  double trimean() const {
    if (x_.empty()) return std::numeric_limits<double>::quiet_NaN();
    std::vector<double> s = x_;
    std::sort(s.begin(), s.end());
    const size_t n = s.size();
    const double q1 = s[n / 4 * 1];
    const double q2 = s[n / 4 * 2];
    const double q3 = s[n / 4 * 3];
    return (q1 + 2 * q2 + q3) / 4;
  }
  double med() const {
    if (x_.empty()) return std::numeric_limits<double>::quiet_NaN();
    std::vector<double> s = x_;
    std::sort(s.begin(), s.end());
    const size_t n = s.size();
    if (n % 2) return s[n / 2];
    return (s[n / 2 - 1] + s[n / 2]) / 2;
  }
  double stddev() const {
    if (x_.size() < 2) return 0;
    const double m = avg();
    double acc = 0;
    for (double v : x_) acc += (v - m) * (v - m);
    return std::sqrt(acc / double(x_.size() - 1)); // sample stddev, as the reference
  }
  const std::vector<double> &samples() const { return x_; }
};
