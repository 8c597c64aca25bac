#pragma once
// Tiny command-line parser for the C++ apps.
// Parity: the reference vendors cwpearson/argparse (thirdparty/argparse/argparse.hpp: add_flag / add_option /
// add_positional / required / help) and cxxopts; this is a self-contained equivalent with the same usage shape.
#include <cstdlib>
#include <functional>
#include <iostream>
#include <sstream>
#include <string>
#include <vector>

namespace stencil {

class ArgParser {
  struct Opt {
    std::vector<std::string> names;
    std::string help;
    bool flag;
    std::function<void(const std::string &)> set;
  };
  struct Pos {
    std::string name, help;
    bool required;
    std::function<void(const std::string &)> set;
  };
  std::string desc_;
  std::vector<Opt> opts_;
  std::vector<Pos> pos_;
  bool help_ = false;

  static std::vector<std::string> split(const std::string &names) {
    std::vector<std::string> r;
    std::stringstream ss(names);
    std::string s;
    while (std::getline(ss, s, ',')) r.push_back(s);
    return r;
  }

public:
  explicit ArgParser(std::string desc) : desc_(std::move(desc)) {}
  ArgParser &flag(bool *dst, const std::string &names, const std::string &help) {
    opts_.push_back({split(names), help, true, [dst](const std::string &) { *dst = true; }});
    return *this;
  }
  template <typename T> ArgParser &option(T *dst, const std::string &names, const std::string &help) {
    opts_.push_back({split(names), help, false, [dst](const std::string &v) {
                       std::stringstream ss(v);
                       ss >> *dst;
                     }});
    return *this;
  }
  ArgParser &option(std::string *dst, const std::string &names, const std::string &help) {
    opts_.push_back({split(names), help, false, [dst](const std::string &v) { *dst = v; }});
    return *this;
  }
  template <typename T> ArgParser &positional(T *dst, const std::string &name, const std::string &help, bool required = false) {
    pos_.push_back({name, help, required, [dst](const std::string &v) {
                      std::stringstream ss(v);
                      ss >> *dst;
                    }});
    return *this;
  }
  std::string usage(const std::string &prog) const {
    std::ostringstream o;
    o << desc_ << "\nusage: " << prog << " [options]";
    for (auto &p : pos_) o << (p.required ? " " : " [") << p.name << (p.required ? "" : "]");
    o << "\n";
    for (auto &p : pos_) o << "  " << p.name << "\t" << p.help << "\n";
    for (auto &op : opts_) {
      o << "  ";
      for (size_t i = 0; i < op.names.size(); ++i) o << (i ? ", " : "") << op.names[i];
      o << (op.flag ? "" : " <v>") << "\t" << op.help << "\n";
    }
    o << "  -h, --help\tshow this help\n";
    return o.str();
  }
  // returns false if the program should exit (help or error)
  bool parse(int argc, char **argv) {
    size_t pi = 0;
    for (int i = 1; i < argc; ++i) {
      std::string a = argv[i];
      if (a == "-h" || a == "--help") {
        std::cout << usage(argv[0]);
        help_ = true;
        return false;
      }
      bool matched = false;
      if (a.size() > 1 && a[0] == '-' && !(a.size() > 1 && (isdigit(a[1]) || a[1] == '.'))) {
        std::string val;
        auto eq = a.find('=');
        std::string key = eq == std::string::npos ? a : a.substr(0, eq);
        for (auto &op : opts_) {
          for (auto &n : op.names)
            if (n == key) {
              matched = true;
              if (op.flag) {
                op.set("");
              } else {
                if (eq != std::string::npos)
                  val = a.substr(eq + 1);
                else if (i + 1 < argc)
                  val = argv[++i];
                else {
                  std::cerr << "missing value for " << key << "\n";
                  return false;
                }
                op.set(val);
              }
              break;
            }
          if (matched) break;
        }
        if (!matched) {
          std::cerr << "unrecognized option " << a << "\n" << usage(argv[0]);
          return false;
        }
      } else {
        if (pi >= pos_.size()) {
          std::cerr << "unexpected positional " << a << "\n";
          return false;
        }
        pos_[pi++].set(a);
      }
    }
    for (size_t k = pi; k < pos_.size(); ++k)
      if (pos_[k].required) {
        std::cerr << "missing required " << pos_[k].name << "\n" << usage(argv[0]);
        return false;
      }
    return true;
  }
  bool need_help() const { return help_; }
};

} // namespace stencil
