// Native fold-file ingestion (include/mmsbm_io.h): the canonical-format fast path of
// Model.get_traintest (src/TrigenicInteractionPredictor.py:321-423).
//
// Per line, like the reference:
//   train  fields = line.strip().split('\t'); genes = fields[0].split('_'); r = int(fields[1])
//   test   fields = re.split(r'\t+', line);   genes = fields[0].split('_'); r = int(fields[1])
//   each gene in file order: first appearance -> next id; uniqueg[id] += 1
//   key = the three ids sorted as decimal strings, joined by '_'; links[key][r] += 1
// Inputs the reference would treat differently from this canonical reading (an exception, a
// negative rating indexing from the end, other line separators of str.splitlines) are not
// guessed at: the parse returns MMSBM_IO_FALLBACK and the Python reader handles them.
#include "mmsbm_io.h"

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <string>
#include <string_view>
#include <unordered_map>
#include <vector>

struct mmsbm_fold {
  std::vector<std::string> names;  // id -> gene name
  std::vector<int32_t> uniqueg;
  std::vector<int32_t> ids[2];     // [E][3] key order
  std::vector<int32_t> counts[2];  // [E][2]
};

namespace {

bool read_file(const char* path, std::string* out) {
  FILE* f = std::fopen(path, "rb");
  if (!f) return false;
  std::fseek(f, 0, SEEK_END);
  const long n = std::ftell(f);
  std::fseek(f, 0, SEEK_SET);
  if (n < 0) {
    std::fclose(f);
    return false;
  }
  out->resize((size_t)n);
  const size_t got = n ? std::fread(&(*out)[0], 1, (size_t)n, f) : 0;
  std::fclose(f);
  return got == (size_t)n;
}

// printable ASCII, TAB and '\n' only: then str.splitlines == split at '\n', and Python's
// whitespace set within a line is {' ', '\t'}
bool canonical_bytes(const std::string& s) {
  for (unsigned char ch : s)
    if (!((ch >= 0x20 && ch < 0x7F) || ch == '\t' || ch == '\n')) return false;
  return true;
}

bool is_ws(char c) { return c == ' ' || c == '\t' || c == '\n'; }

// Python int(text) restricted to: whitespace, optional sign, ASCII digits, whitespace.  Returns
// false for anything else (underscores, empty, overflow-sized) -> fallback.
bool py_int(std::string_view t, long* v) {
  size_t a = 0, b = t.size();
  while (a < b && is_ws(t[a])) ++a;
  while (b > a && is_ws(t[b - 1])) --b;
  if (a == b) return false;
  bool neg = false;
  if (t[a] == '+' || t[a] == '-') {
    neg = t[a] == '-';
    ++a;
  }
  if (a == b || b - a > 9) return false;
  long x = 0;
  for (size_t i = a; i < b; ++i) {
    if (t[i] < '0' || t[i] > '9') return false;
    x = x * 10 + (t[i] - '0');
  }
  *v = neg ? -x : x;
  return true;
}

struct KeyHash {
  size_t operator()(const uint64_t& k) const { return std::hash<uint64_t>()(k * 0x9E3779B97F4A7C15ull); }
};

struct SvHash {
  size_t operator()(std::string_view s) const { return std::hash<std::string_view>()(s); }
};

class Reader {
 public:
  explicit Reader(mmsbm_fold* f) : f_(f) {}

  // which: 0 train (strip + split('\t')), 1 test (re.split(r'\t+') on the unstripped line)
  bool parse(const std::string& text, int which) {
    size_t pos = 0;
    const size_t n = text.size();
    const size_t lines = (size_t)std::count(text.begin(), text.end(), '\n') + 1;
    links_[which].reserve(lines);
    f_->ids[which].reserve(3 * lines);
    f_->counts[which].reserve(2 * lines);
    if (gid_.empty()) gid_.reserve(lines / 4 + 16);
    while (pos < n) {
      size_t end = text.find('\n', pos);
      const size_t stop = end == std::string::npos ? n : end + 1;  // readlines keeps '\n'
      std::string_view line(text.data() + pos, stop - pos);
      pos = stop;
      std::string_view genes, rfield;
      if (which == 0) {
        size_t a = 0, b = line.size();
        while (a < b && is_ws(line[a])) ++a;
        while (b > a && is_ws(line[b - 1])) --b;
        std::string_view s = line.substr(a, b - a);
        const size_t t1 = s.find('\t');
        if (t1 == std::string_view::npos) return false;  // fields[1] -> IndexError
        genes = s.substr(0, t1);
        const size_t t2 = s.find('\t', t1 + 1);
        rfield = s.substr(t1 + 1, t2 == std::string_view::npos ? std::string_view::npos : t2 - t1 - 1);
      } else {
        const size_t t1 = line.find('\t');
        if (t1 == std::string_view::npos) return false;
        genes = line.substr(0, t1);
        size_t r0 = t1;
        while (r0 < line.size() && line[r0] == '\t') ++r0;
        const size_t t2 = line.find('\t', r0);
        rfield = line.substr(r0, t2 == std::string_view::npos ? std::string_view::npos : t2 - r0);
        if (r0 == line.size()) return false;  // re.split leaves '' last: int('') ValueError
      }
      long r = 0;
      if (!py_int(rfield, &r) || (r != 0 && r != 1)) return false;
      // exactly three genes
      const size_t u1 = genes.find('_');
      if (u1 == std::string_view::npos) return false;
      const size_t u2 = genes.find('_', u1 + 1);
      if (u2 == std::string_view::npos || genes.find('_', u2 + 1) != std::string_view::npos)
        return false;
      const std::string_view g[3] = {genes.substr(0, u1), genes.substr(u1 + 1, u2 - u1 - 1),
                                     genes.substr(u2 + 1)};
      int32_t id[3];
      for (int i = 0; i < 3; ++i) {
        auto it = gid_.find(g[i]);  // views into the file texts, alive for the whole parse
        if (it == gid_.end()) {
          id[i] = (int32_t)f_->names.size();
          f_->names.emplace_back(g[i]);
          f_->uniqueg.push_back(0);
          dec_.push_back(std::to_string(id[i]));
          gid_.emplace(g[i], id[i]);
        } else {
          id[i] = it->second;
        }
        f_->uniqueg[id[i]] += 1;
      }
      key_order(id);
      const uint64_t k = ((uint64_t)(uint32_t)id[0] << 42) ^ ((uint64_t)(uint32_t)id[1] << 21) ^
                         (uint64_t)(uint32_t)id[2];
      if (id[0] >= (1 << 21) || id[1] >= (1 << 21) || id[2] >= (1 << 21)) return false;
      auto& rows = links_[which];
      auto it = rows.find(k);
      size_t row;
      if (it == rows.end()) {
        row = f_->counts[which].size() / 2;
        rows.emplace(k, row);
        f_->ids[which].insert(f_->ids[which].end(), id, id + 3);
        f_->counts[which].push_back(0);
        f_->counts[which].push_back(0);
      } else {
        row = it->second;
      }
      f_->counts[which][row * 2 + r] += 1;
    }
    return true;
  }

 private:
  // the three ids in the reference's key order: sorted as decimal strings ('10' < '2')
  void key_order(int32_t* v) const {
    auto lt = [&](int32_t x, int32_t y) { return dec_[x] < dec_[y]; };
    if (lt(v[1], v[0])) std::swap(v[0], v[1]);
    if (lt(v[2], v[1])) std::swap(v[1], v[2]);
    if (lt(v[1], v[0])) std::swap(v[0], v[1]);
  }

  mmsbm_fold* f_;
  std::unordered_map<std::string_view, int32_t, SvHash> gid_;
  std::vector<std::string> dec_;  // id -> its decimal string
  std::unordered_map<uint64_t, size_t, KeyHash> links_[2];
};

}  // namespace

extern "C" {

int mmsbm_fold_parse(const char* train_path, const char* test_path, mmsbm_fold** out) {
  if (!train_path || !test_path || !out) return MMSBM_IO_INVALID;
  *out = nullptr;
  std::string tr, te;
  if (!read_file(train_path, &tr) || !read_file(test_path, &te)) return MMSBM_IO_FALLBACK;
  if (!canonical_bytes(tr) || !canonical_bytes(te)) return MMSBM_IO_FALLBACK;
  auto* f = new mmsbm_fold();
  Reader rd(f);
  if (!rd.parse(tr, 0) || !rd.parse(te, 1)) {
    delete f;
    return MMSBM_IO_FALLBACK;
  }
  *out = f;
  return MMSBM_IO_OK;
}

int mmsbm_fold_sizes(const mmsbm_fold* f, int64_t* P, int64_t* E_train, int64_t* E_test,
                     int64_t* names_bytes) {
  if (!f || !P || !E_train || !E_test || !names_bytes) return MMSBM_IO_INVALID;
  *P = (int64_t)f->names.size();
  *E_train = (int64_t)f->counts[0].size() / 2;
  *E_test = (int64_t)f->counts[1].size() / 2;
  int64_t nb = 0;
  for (const auto& s : f->names) nb += (int64_t)s.size() + 1;
  *names_bytes = nb;
  return MMSBM_IO_OK;
}

int mmsbm_fold_export(const mmsbm_fold* f, char* names, int32_t* uniqueg, int32_t* train_ids,
                      int32_t* train_counts, int32_t* test_ids, int32_t* test_counts) {
  if (!f) return MMSBM_IO_INVALID;
  if (names) {
    for (const auto& s : f->names) {
      std::memcpy(names, s.data(), s.size());
      names += s.size();
      *names++ = '\0';
    }
  }
  auto put = [](int32_t* dst, const std::vector<int32_t>& v) {
    if (dst && !v.empty()) std::memcpy(dst, v.data(), v.size() * sizeof(int32_t));
  };
  put(uniqueg, f->uniqueg);
  put(train_ids, f->ids[0]);
  put(train_counts, f->counts[0]);
  put(test_ids, f->ids[1]);
  put(test_counts, f->counts[1]);
  return MMSBM_IO_OK;
}

void mmsbm_fold_free(mmsbm_fold* f) { delete f; }

}  // extern "C"
