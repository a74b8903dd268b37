// io.cpp -- rating-file reader and model snapshots, on top of the C ABI.
//
//  * mf_read_ratings: the reference's input, env.readCsvFile[(Int, Int, Double)](path)
//    (DSGDforMF.scala:72; Flink's defaults: "\n" lines, "," fields), and MovieLens u.data
//    (tab-separated user, item, rating, timestamp).  The file is memory-mapped, cut at line
//    boundaries into one chunk per thread, counted, then parsed in parallel into the caller's
//    arrays.  Fields after the third are ignored; a malformed line is an MF_ERR_INVALID naming
//    the line, as Flink's CSV parser fails the job.
//  * mf_save_model / mf_load_model: the role of the reference's TemporaryPath persistence
//    (DSGDforMF.scala:291-296, 330-333, 346-349): a binary snapshot of both factor sides (ids
//    ascending, f64) and the superstep counter, so a fit can be resumed or its model reused.
#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <charconv>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "common.hpp"
#include "mfhip.h"

namespace mfhip {
namespace {

struct MappedFile {
  const char* data = nullptr;
  size_t size = 0;
  int fd = -1;
  explicit MappedFile(const char* path) {
    fd = ::open(path, O_RDONLY);
    if (fd < 0) fail(MF_ERR_INVALID, std::string("cannot open ") + path);
    struct stat st;
    if (fstat(fd, &st) != 0) fail(MF_ERR_INVALID, std::string("cannot stat ") + path);
    size = static_cast<size_t>(st.st_size);
    if (size > 0) {
      void* p = mmap(nullptr, size, PROT_READ, MAP_PRIVATE, fd, 0);
      if (p == MAP_FAILED) fail(MF_ERR_INVALID, std::string("cannot map ") + path);
      data = static_cast<const char*>(p);
    }
  }
  ~MappedFile() {
    if (data) munmap(const_cast<char*>(data), size);
    if (fd >= 0) ::close(fd);
  }
};

bool blank(const char* b, const char* e) {
  for (; b < e; ++b)
    if (*b != ' ' && *b != '\t' && *b != '\r') return false;
  return true;
}

// One "user<d>item<d>rating[<d>...]" line; d = delim, or any run of spaces / tabs / commas when
// delim == 0.
bool parse_line(const char* b, const char* e, char delim, int32_t& u, int32_t& i, double& r) {
  auto sep = [&](char c) { return delim ? c == delim : (c == ' ' || c == '\t' || c == ','); };
  auto skip_sep = [&](const char*& p) {
    if (p >= e || !sep(*p)) return false;
    ++p;
    if (!delim) while (p < e && sep(*p)) ++p;
    return true;
  };
  auto skip_ws = [&](const char*& p) { while (p < e && (*p == ' ' || *p == '\r') && !sep(*p)) ++p; };
  const char* p = b;
  skip_ws(p);
  auto a = std::from_chars(p, e, u);
  if (a.ec != std::errc()) return false;
  p = a.ptr;
  skip_ws(p);
  if (!skip_sep(p)) return false;
  skip_ws(p);
  a = std::from_chars(p, e, i);
  if (a.ec != std::errc()) return false;
  p = a.ptr;
  skip_ws(p);
  if (!skip_sep(p)) return false;
  skip_ws(p);
  auto c = std::from_chars(p, e, r);
  if (c.ec != std::errc()) return false;
  p = c.ptr;
  skip_ws(p);
  return p >= e || sep(*p);
}

constexpr char kMagic[8] = {'M', 'F', 'H', 'I', 'P', 'S', 'N', '1'};

void check(int st) {
  if (st != MF_OK) fail(st, mf_last_error());
}

}  // namespace
}  // namespace mfhip

using namespace mfhip;

extern "C" {

int mf_read_ratings(const char* path, char delim, int32_t skip_lines, int32_t* users, int32_t* items,
                    double* ratings, int64_t cap, int64_t* n_out) {
  return guarded([&] {
    MF_REQUIRE(path && n_out && skip_lines >= 0, "bad argument");
    MappedFile f(path);
    const char* b = f.data;
    const char* end = f.data + f.size;
    for (int32_t s = 0; s < skip_lines && b < end; ++s) {
      const char* nl = static_cast<const char*>(std::memchr(b, '\n', static_cast<size_t>(end - b)));
      b = nl ? nl + 1 : end;
    }
    const int T = host_threads();
    std::vector<const char*> cut(T + 1, end);
    cut[0] = b;
    for (int t = 1; t < T; ++t) {
      const char* p = b + static_cast<size_t>(end - b) * t / T;
      if (p < cut[t - 1]) p = cut[t - 1];
      const char* nl = p < end ? static_cast<const char*>(std::memchr(p, '\n', static_cast<size_t>(end - p))) : nullptr;
      cut[t] = nl ? nl + 1 : end;
    }
    // pass 1: non-blank lines per chunk (and the chunk's first line number, for errors)
    std::vector<int64_t> cnt(T, 0), lines(T, 0);
    parallel_tasks(T, [&](int64_t t) {
      for (const char* p = cut[t]; p < cut[t + 1];) {
        const char* nl = static_cast<const char*>(std::memchr(p, '\n', static_cast<size_t>(cut[t + 1] - p)));
        const char* e = nl ? nl : cut[t + 1];
        if (!blank(p, e)) cnt[t]++;
        lines[t]++;
        p = nl ? nl + 1 : cut[t + 1];
      }
    });
    std::vector<int64_t> base(T + 1, 0), line0(T + 1, skip_lines + 1);
    for (int t = 0; t < T; ++t) {
      base[t + 1] = base[t] + cnt[t];
      line0[t + 1] = line0[t] + lines[t];
    }
    *n_out = base[T];
    if (!users) return;  // count only
    MF_REQUIRE(items && ratings, "null output arrays");
    MF_REQUIRE(cap >= base[T], "output capacity below the record count");
    std::vector<int64_t> bad(T, -1);
    parallel_tasks(T, [&](int64_t t) {
      int64_t x = base[t], ln = line0[t];
      for (const char* p = cut[t]; p < cut[t + 1]; ++ln) {
        const char* nl = static_cast<const char*>(std::memchr(p, '\n', static_cast<size_t>(cut[t + 1] - p)));
        const char* e = nl ? nl : cut[t + 1];
        if (!blank(p, e)) {
          if (!parse_line(p, e, delim, users[x], items[x], ratings[x])) { bad[t] = ln; return; }
          ++x;
        }
        p = nl ? nl + 1 : cut[t + 1];
      }
    });
    for (int t = 0; t < T; ++t)
      if (bad[t] >= 0) fail(MF_ERR_INVALID, std::string(path) + ": cannot parse line " + std::to_string(bad[t]) +
                                                " as (Int, Int, Double)");
  });
}

int mf_save_model(mf_ctx* ctx, const char* path) {
  return guarded([&] {
    MF_REQUIRE(ctx && path, "null argument");
    mf_params P;
    check(mf_get_params(ctx, &P));
    const int32_t k = P.num_factors;
    int64_t nu = 0, ni = 0, step = 0;
    check(mf_num_factors(ctx, MF_SIDE_USER, &nu));
    check(mf_num_factors(ctx, MF_SIDE_ITEM, &ni));
    check(mf_dsgd_superstep(ctx, &step));
    std::vector<int32_t> ids;
    std::vector<double> vecs;
    FILE* f = std::fopen(path, "wb");
    MF_REQUIRE(f, std::string("cannot create ") + path);
    bool ok = std::fwrite(kMagic, 1, 8, f) == 8 && std::fwrite(&k, 4, 1, f) == 1 &&
              std::fwrite(&step, 8, 1, f) == 1 && std::fwrite(&nu, 8, 1, f) == 1 && std::fwrite(&ni, 8, 1, f) == 1;
    for (int side = 0; side < 2 && ok; ++side) {
      const int64_t n = side == MF_SIDE_USER ? nu : ni;
      ids.resize(n);
      vecs.resize(static_cast<size_t>(n) * k);
      int64_t got = 0;
      if (n > 0) {
        const int st = mf_get_factors(ctx, side, ids.data(), vecs.data(), n, &got);
        if (st != MF_OK) { std::fclose(f); fail(st, mf_last_error()); }
      }
      ok = std::fwrite(ids.data(), 4, n, f) == static_cast<size_t>(n) &&
           std::fwrite(vecs.data(), 8, vecs.size(), f) == vecs.size();
    }
    ok = (std::fclose(f) == 0) && ok;
    MF_REQUIRE(ok, std::string("write failed: ") + path);
  });
}

int mf_load_model(mf_ctx* ctx, const char* path, int64_t* superstep_out) {
  return guarded([&] {
    MF_REQUIRE(ctx && path, "null argument");
    mf_params P;
    check(mf_get_params(ctx, &P));
    FILE* f = std::fopen(path, "rb");
    MF_REQUIRE(f, std::string("cannot open ") + path);
    char magic[8];
    int32_t k = 0;
    int64_t step = 0, n[2] = {0, 0};
    bool ok = std::fread(magic, 1, 8, f) == 8 && std::memcmp(magic, kMagic, 8) == 0 &&
              std::fread(&k, 4, 1, f) == 1 && std::fread(&step, 8, 1, f) == 1 && std::fread(n, 8, 2, f) == 2;
    if (!ok || k != P.num_factors || n[0] < 0 || n[1] < 0 || step < 0) {
      std::fclose(f);
      fail(MF_ERR_INVALID, std::string(path) + ": not an mfhip snapshot of rank " + std::to_string(P.num_factors));
    }
    for (int side = 0; side < 2; ++side) {
      std::vector<int32_t> ids(n[side]);
      std::vector<double> vecs(static_cast<size_t>(n[side]) * k);
      ok = std::fread(ids.data(), 4, ids.size(), f) == ids.size() &&
           std::fread(vecs.data(), 8, vecs.size(), f) == vecs.size();
      if (!ok) { std::fclose(f); fail(MF_ERR_INVALID, std::string(path) + ": truncated snapshot"); }
      const int st = mf_set_factors(ctx, side, ids.data(), vecs.data(), n[side]);
      if (st != MF_OK) { std::fclose(f); fail(st, mf_last_error()); }
    }
    std::fclose(f);
    if (superstep_out) *superstep_out = step;
  });
}

}  // extern "C"
