// .ini / .dataset reader: the subset of TIniFile (reference source/IniObjects.f90)
// that CMB dataset files use, plus File%LoadTxt (source/FileUtils.f90).
#include <sys/stat.h>

#include <cctype>
#include <cstring>
#include <fstream>
#include <sstream>

#include "common.h"

namespace cmamd {

static std::string trim(const std::string &s) {
    size_t a = 0, b = s.size();
    while (a < b && std::isspace((unsigned char)s[a])) a++;
    while (b > a && std::isspace((unsigned char)s[b - 1])) b--;
    return s.substr(a, b - a);
}

std::vector<std::string> split_ws(const std::string &s) {
    std::vector<std::string> out;
    std::istringstream is(s);
    std::string t;
    while (is >> t) out.push_back(t);
    return out;
}

std::string dirname_of(const std::string &path) {
    size_t p = path.find_last_of('/');
    return p == std::string::npos ? std::string() : path.substr(0, p + 1);
}

bool file_exists(const std::string &path) {
    struct stat st;
    return stat(path.c_str(), &st) == 0 && S_ISREG(st.st_mode);
}

void Ini::add_line(const std::string &raw, bool only_if_undefined) {
    std::string line = trim(raw);
    if (line.empty() || line[0] == '#') return;
    size_t eq = line.find('=');
    if (eq == std::string::npos) return;
    std::string k = trim(line.substr(0, eq)), v = trim(line.substr(eq + 1));
    if (k.empty()) return;
    // first definition wins (TNameValueList ignoreDuplicates); only_if_undefined
    // is the same rule for DEFAULT() files
    (void)only_if_undefined;
    if (!kv_.count(k)) kv_[k] = v;
}

void Ini::open_rec(const std::string &fname, bool only_if_undefined, int depth) {
    if (depth > 16) fail(CMBL_ERR_FORMAT, "ini: INCLUDE/DEFAULT nesting too deep at %s", fname.c_str());
    std::ifstream f(fname);
    if (!f) fail(CMBL_ERR_IO, "ini file not found: %s", fname.c_str());
    std::vector<std::string> includes, defaults;
    std::string line;
    while (std::getline(f, line)) {
        std::string t = trim(line);
        if (t == "END") break;
        if (t.rfind("INCLUDE(", 0) == 0 || t.rfind("DEFAULT(", 0) == 0) {
            size_t close = t.find(')');
            if (close == std::string::npos) fail(CMBL_ERR_FORMAT, "ini: bad include line in %s", fname.c_str());
            (t[0] == 'I' ? includes : defaults).push_back(t.substr(8, close - 8));
            continue;
        }
        add_line(t, only_if_undefined);
    }
    auto resolve = [&](const std::string &n) {
        if (!n.empty() && n[0] == '/') return n;
        std::string cand = dirname_of(fname) + n;
        return file_exists(cand) ? cand : n;
    };
    for (auto &i : includes) open_rec(resolve(i), only_if_undefined, depth + 1);
    for (auto &d : defaults) open_rec(resolve(d), true, depth + 1);
}

void Ini::open(const std::string &filename) {
    filename_ = filename;
    open_rec(filename, false, 0);
}

void Ini::override_text(const char *text) {
    if (!text) return;
    std::istringstream is(text);
    std::string line;
    while (std::getline(is, line)) {
        line = trim(line);
        size_t eq = line.find('=');
        if (line.empty() || line[0] == '#' || eq == std::string::npos) continue;
        kv_[trim(line.substr(0, eq))] = trim(line.substr(eq + 1));   // Override replaces
    }
}

std::string Ini::str(const std::string &key, const std::string &def) const {
    auto it = kv_.find(key);
    return it == kv_.end() ? def : it->second;
}

std::string Ini::str_required(const std::string &key) const {
    auto it = kv_.find(key);
    if (it == kv_.end() || it->second.empty())
        fail(CMBL_ERR_FORMAT, "%s: required key '%s' missing", filename_.c_str(), key.c_str());
    return it->second;
}

std::string Ini::relative_filename(const std::string &key, bool required) const {
    return resolve_path(required ? str_required(key) : str(key));
}

std::string Ini::resolve_path(std::string v) const {
    if (v.empty()) return v;
    // %DATASETDIR% / %LOCALDIR% (settings.f90:183-184): resolve against the
    // environment override or leave for the relative rule below
    const char *dd = std::getenv("COSMOMC_DATASETDIR");
    size_t p;
    if ((p = v.find("%DATASETDIR%")) != std::string::npos) v.replace(p, 12, dd ? dd : "data/");
    if ((p = v.find("%LOCALDIR%")) != std::string::npos) v.replace(p, 10, "./");
    if (v[0] == '/') return v;
    std::string cand = dirname_of(filename_) + v;
    if (file_exists(cand)) return cand;
    return v;
}

std::vector<std::vector<double>> load_txt(const std::string &path) {
    std::ifstream f(path);
    if (!f) fail(CMBL_ERR_IO, "cannot read %s", path.c_str());
    std::vector<std::vector<double>> rows;
    std::string line;
    size_t ncol = 0;
    while (std::getline(f, line)) {
        std::string t = trim(line);
        if (t.empty() || t[0] == '#') continue;
        std::vector<double> r;
        const char *s = t.c_str();
        char *end;
        while (*s) {
            while (*s && (std::isspace((unsigned char)*s) || *s == ',')) s++;
            if (!*s) break;
            double v = std::strtod(s, &end);
            if (end == s) fail(CMBL_ERR_FORMAT, "%s: non-numeric entry", path.c_str());
            r.push_back(v);
            s = end;
        }
        if (ncol == 0) ncol = r.size();
        if (r.size() != ncol) fail(CMBL_ERR_FORMAT, "%s: ragged rows", path.c_str());
        rows.push_back(std::move(r));
    }
    return rows;
}

}  // namespace cmamd
