// clip_csv.cpp - runtime loader of the reference's per-clip CSV quadruple (host code, part of libhumenv.so).
//
// Replaces LowLevelHumanoidEnv.__init__'s table loading (/root/reference/low_level_env.py:58-70:
// pd.read_csv of <clip>JointPosRad.csv, JointSpeedRadSec.csv, JointPosRadRelative.csv, JointVecFromHip.csv).
// Values are parsed with pandas' default C-engine float converter (float_precision=None = "high",
// pandas/_libs/src/parser/tokenizer.c precise_xstrtod: up to 17 significant digits accumulated as
// number * 10 + digit in double, then one multiply / divide by an exactly-rounded power of ten), so every table
// entry is bit-identical to what the reference env reads with DataFrame.iloc - pandas' parser is not
// correctly rounded, so strtod would differ in the last bit for some entries.  Columns are selected by header
// name in the fixed order of include/humanoid_env.h (hum_set_clip).
#include <cerrno>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/humanoid_env.h"

// hum_last_error()'s message (humanoid_env.hip)
void hum_internal_set_error(const char* msg);

namespace {

struct ErrSink {
    ErrSink& operator=(const std::string& m) { hum_internal_set_error(m.c_str()); return *this; }
} g_csv_err;

const char* kJointCols[14] = {"rightHipX", "rightHipY", "rightHipZ", "rightKnee", "leftHipX", "leftHipY", "leftHipZ",
                              "leftKnee", "rightShoulderX", "rightShoulderY", "rightElbow", "leftShoulderX",
                              "leftShoulderY", "leftElbow"};
const char* kEpParts[9] = {"LeftLeg", "LeftFoot", "RightLeg", "RightFoot", "Head", "LeftForeArm", "LeftHand",
                           "RightForeArm", "RightHand"};
const char* kSuffix[4] = {"JointPosRad", "JointSpeedRadSec", "JointPosRadRelative", "JointVecFromHip"};


// pandas precise_xstrtod (decimal '.', sci 'e'/'E', no thousands separator)
double pandas_xstrtod(const char* p, const char** end, bool* ok) {
    struct Pow10 {   // pandas' table of exactly-rounded powers of ten (thread-safe static init)
        double v[309];
        Pow10() { for (int i = 0; i <= 308; i++) v[i] = std::strtod(("1e" + std::to_string(i)).c_str(), nullptr); }
    };
    static const Pow10 P10;
    const double* e = P10.v;
    *ok = true;
    while (*p == ' ' || *p == '\t') p++;
    bool neg = false;
    if (*p == '-') { neg = true; p++; }
    else if (*p == '+') p++;
    double number = 0.;
    int exponent = 0, num_digits = 0, num_decimals = 0;
    const int max_digits = 17;
    while (*p >= '0' && *p <= '9') {
        if (num_digits < max_digits) {
            number = number * 10. + (*p - '0');
            num_digits++;
        } else {
            ++exponent;
        }
        p++;
    }
    if (*p == '.') {
        p++;
        while (num_digits < max_digits && *p >= '0' && *p <= '9') {
            number = number * 10. + (*p - '0');
            p++;
            num_digits++;
            num_decimals++;
        }
        if (num_digits >= max_digits)
            while (*p >= '0' && *p <= '9') ++p;
        exponent -= num_decimals;
    }
    if (num_digits == 0) { *ok = false; *end = p; return 0.0; }
    if (neg) number = -number;
    if (*p == 'e' || *p == 'E') {
        const char* q = p + 1;
        bool eneg = false;
        if (*q == '-') { eneg = true; q++; }
        else if (*q == '+') q++;
        if (*q >= '0' && *q <= '9') {
            int n = 0;
            while (*q >= '0' && *q <= '9') { n = n * 10 + (*q - '0'); q++; }
            exponent += eneg ? -n : n;
            p = q;
        }
    }
    if (exponent > 308) { *ok = false; *end = p; return HUGE_VAL; }
    else if (exponent > 0) number *= e[exponent];
    else if (exponent < -308) {
        if (exponent < -616) number = 0.;
        else { number /= e[-308 - exponent]; number /= e[308]; }
    } else number /= e[-exponent];
    *end = p;
    return number;
}

bool read_file(const std::string& path, std::string& out) {
    FILE* f = std::fopen(path.c_str(), "rb");
    if (!f) { g_csv_err = "cannot open " + path; return false; }
    std::fseek(f, 0, SEEK_END);
    const long n = std::ftell(f);
    std::fseek(f, 0, SEEK_SET);
    out.resize(n > 0 ? (size_t)n : 0);
    const size_t got = n > 0 ? std::fread(&out[0], 1, (size_t)n, f) : 0;
    std::fclose(f);
    if ((long)got != n) { g_csv_err = "short read " + path; return false; }
    return true;
}

// parse one CSV (header line + rows of floats); returns the requested columns row-major
bool parse_csv(const std::string& path, const std::vector<std::string>& cols, std::vector<double>& out, int& rows) {
    std::string txt;
    if (!read_file(path, txt)) return false;
    size_t pos = 0;
    auto next_line = [&](std::string& line) -> bool {
        if (pos >= txt.size()) return false;
        size_t e = txt.find('\n', pos);
        if (e == std::string::npos) e = txt.size();
        line.assign(txt, pos, e - pos);
        if (!line.empty() && line.back() == '\r') line.pop_back();
        pos = e + 1;
        return true;
    };
    std::string line;
    if (!next_line(line)) { g_csv_err = path + ": empty"; return false; }
    std::vector<std::string> header;
    {
        size_t s = 0;
        while (true) {
            size_t c = line.find(',', s);
            header.push_back(line.substr(s, c == std::string::npos ? std::string::npos : c - s));
            if (c == std::string::npos) break;
            s = c + 1;
        }
    }
    std::vector<int> idx;
    for (const auto& c : cols) {
        int k = -1;
        for (size_t j = 0; j < header.size(); j++)
            if (header[j] == c) k = (int)j;
        if (k < 0) { g_csv_err = path + ": missing column " + c; return false; }
        idx.push_back(k);
    }
    out.clear();
    rows = 0;
    std::vector<double> vals;
    while (next_line(line)) {
        if (line.empty()) continue;
        vals.clear();
        const char* p = line.c_str();
        while (true) {
            const char* e;
            bool ok;
            const double v = pandas_xstrtod(p, &e, &ok);
            if (!ok) { g_csv_err = path + ": bad number in row " + std::to_string(rows); return false; }
            vals.push_back(v);
            while (*e == ' ' || *e == '\t') e++;
            if (*e == ',') { p = e + 1; continue; }
            if (*e == '\0') break;
            g_csv_err = path + ": unexpected character in row " + std::to_string(rows);
            return false;
        }
        if (vals.size() != header.size()) { g_csv_err = path + ": ragged row " + std::to_string(rows); return false; }
        for (int k : idx) out.push_back(vals[(size_t)k]);
        rows++;
    }
    return true;
}

bool parse_clip(const char* dir, const char* name, std::vector<double> t[4], int n[4]) {
    if (!dir || !name) { g_csv_err = "null argument"; return false; }
    std::vector<std::string> jc(kJointCols, kJointCols + 14), ec;
    for (const char* part : kEpParts)
        for (const char* ax : {"X", "Y", "Z"}) ec.push_back(std::string(part) + "_" + ax + "position");
    for (int k = 0; k < 4; k++) {
        const std::string path = std::string(dir) + "/" + name + kSuffix[k] + ".csv";
        if (!parse_csv(path, k == 3 ? ec : jc, t[k], n[k])) return false;
    }
    return true;
}

}  // namespace

extern "C" {

int hum_clip_csv_sizes(const char* dir, const char* name, int32_t* sizes4) {
    std::vector<double> t[4];
    int n[4];
    if (!sizes4 || !parse_clip(dir, name, t, n)) return HUM_ERR_ARG;
    for (int k = 0; k < 4; k++) sizes4[k] = n[k];
    return HUM_OK;
}

int hum_clip_csv_parse(const char* dir, const char* name, double* pos, double* vel, double* rel, double* ep) {
    std::vector<double> t[4];
    int n[4];
    if (!pos || !vel || !rel || !ep || !parse_clip(dir, name, t, n)) return HUM_ERR_ARG;
    double* dst[4] = {pos, vel, rel, ep};
    for (int k = 0; k < 4; k++) std::memcpy(dst[k], t[k].data(), t[k].size() * sizeof(double));
    return HUM_OK;
}

int hum_load_clip_csv(hum_env* env, int32_t clip_id, const char* dir, const char* name) {
    std::vector<double> t[4];
    int n[4];
    if (!env || !parse_clip(dir, name, t, n)) return HUM_ERR_ARG;
    return hum_set_clip(env, clip_id, t[0].data(), n[0], t[1].data(), n[1], t[2].data(), n[2], t[3].data(), n[3]);
}

}  // extern "C"
