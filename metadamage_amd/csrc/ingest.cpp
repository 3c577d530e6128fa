// ingest.cpp — memory-mapped, multi-threaded reader of metadamage count
// tables (include/mdingest.h).
//
// mdi_open maps the file, detects the format and cuts it at line boundaries
// into one chunk per thread, counting each chunk's rows (memchr over
// newlines).  mdi_parse_into then lets every thread parse its chunk straight
// into the caller's column arrays at the chunk's row offset -- no growth, no
// concatenation, no copy -- interning the string columns per chunk (a taxon's
// rows repeat its name, so the previous row's string is tried first); the
// chunks' string tables are merged in file order and the codes rewritten in
// parallel.
#include "../../include/mdingest.h"

#include <fcntl.h>
#include <sched.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <string_view>
#include <condition_variable>
#include <deque>
#include <mutex>
#include <thread>
#include <unordered_map>
#include <vector>

namespace {

thread_local char g_err[512] = "";

int fail(int code, const char* fmt, long a = 0, long b = 0) {
  std::snprintf(g_err, sizeof(g_err), fmt, a, b);
  return code;
}

struct LocalStrings {
  std::vector<std::string_view> uniq;
  std::unordered_map<std::string_view, int32_t> ids;
  std::string_view last;
  int32_t last_id = -1;
  int32_t add(std::string_view s) {
    if (last_id >= 0 && s == last) return last_id;
    auto it = ids.find(s);
    int32_t id;
    if (it == ids.end()) {
      id = (int32_t)uniq.size();
      uniq.push_back(s);
      ids.emplace(s, id);
    } else {
      id = it->second;
    }
    last = s;
    last_id = id;
    return id;
  }
};

struct Chunk {
  const char* begin = nullptr;
  const char* end = nullptr;
  std::string tail;  // the file's last line when it lacks a newline, with one
  int64_t row0 = 0, rows = 0;  // rows: non-blank lines
  LocalStrings str[3];
  int err = 0;
  long bad_row = 0;
  int bad_col = 0;
};

}  // namespace

struct mdi_table {
  void* map = nullptr;
  size_t size = 0;
  const char* data = nullptr;  // first row (after a header)
  long first_line = 1;
  int format = 22;
  int64_t rows = 0;
  bool parsed = false;
  std::vector<Chunk> chunks;
  std::vector<std::string> strings[3];
};

namespace {

// The scanners below take no end pointer: every line they see ends in '\n'
// (parse_chunk hands a last line without one over as a copy with it appended),
// and none of them moves past a '\n', so the newline is the sentinel.  lim
// bounds the bytes that may be READ (the mapping, or the padded copy): an
// integer with 8 readable bytes ahead is converted 8 digits at a time (SWAR),
// which spares the digit loop's branch per digit and its mispredicted exit.
inline bool parse_int(const char*& p, const char* lim, int64_t* v) {
  bool neg = false;
  if (*p == '-' || *p == '+') {
    neg = *p == '-';
    ++p;
  }
  const char* s = p;
  int64_t x = 0;
  if (lim - p >= 8) {
    uint64_t w;
    std::memcpy(&w, p, 8);
    const uint64_t t = w ^ 0x3030303030303030ull;  // digits -> 0..9
    // a byte is a non-digit iff its high nibble is set, or adding 6 sets it
    // (carries only leave the first non-digit byte, upward: never read)
    const uint64_t nd = (t | (t + 0x0606060606060606ull)) & 0xF0F0F0F0F0F0F0F0ull;
    const int len = nd ? __builtin_ctzll(nd) >> 3 : 8;
    if (len > 0) {
      uint64_t y = t << (8 * (8 - len));  // the len digits right-aligned, first digit most significant
      y = (y * 10 + (y >> 8)) & 0x00FF00FF00FF00FFull;
      y = (y * 100 + (y >> 16)) & 0x0000FFFF0000FFFFull;
      y = (y * 10000 + (y >> 32)) & 0xFFFFFFFFull;
      x = (int64_t)y;
      p += len;
    }
    if (len == 8)
      while ((unsigned)(*p - '0') < 10u) {
        x = x * 10 + (*p - '0');
        ++p;
      }
  } else {
    while ((unsigned)(*p - '0') < 10u) {
      x = x * 10 + (*p - '0');
      ++p;
    }
  }
  if (p == s) return false;
  if (*p == '.') {  // tolerate a float rendering of an integer ("12.0")
    ++p;
    while (*p == '0') ++p;
    if ((unsigned)(*p - '0') < 10u) return false;
  }
  *v = neg ? -x : x;
  return true;
}

inline std::string_view field(const char*& p) {
  const char* s = p;
  while (*p != '\t' && *p != '\n' && *p != '\r') ++p;
  return std::string_view(s, (size_t)(p - s));
}

// a string field, interned: a row repeating the previous row's value (a
// taxon's 30 rows) is matched in place without scanning for its end
inline int32_t intern(const char*& p, const char* lim, LocalStrings& ls) {
  const size_t n = ls.last.size();
  if (ls.last_id >= 0 && (size_t)(lim - p) > n && std::memcmp(p, ls.last.data(), n) == 0) {
    const char d = p[n];
    if (d == '\t' || d == '\n' || d == '\r') {
      p += n;
      return ls.last_id;
    }
  }
  return ls.add(field(p));
}

inline bool tab(const char*& p) {
  if (*p == '\t') {
    ++p;
    return true;
  }
  return false;
}

int64_t count_rows(const char* p, const char* end) {
  int64_t n = 0;
  while (p < end) {
    const char* nl = (const char*)memchr(p, '\n', (size_t)(end - p));
    const char* le = nl ? nl : end;
    if (le > p && !(le - p == 1 && *p == '\r')) ++n;  // non-blank line
    p = nl ? nl + 1 : end;
  }
  return n;
}

struct Out {
  int64_t *tax_id, *nal, *pos, *counts;
  int32_t* code[3];
  int64_t rows;
  const char* map_end;  // readable bytes of the mapping end here
};

// one line [p, its '\n'] into row r; false on a malformed field (col set)
inline bool parse_line(const char*& p, const char* lim, int format, const Out& o, Chunk* c, int64_t r, int& col) {
  col = 0;
  int64_t tid, nal, pos;
  int32_t name = 0, rank = 0;
  if (!parse_int(p, lim, &tid) || !tab(p)) return false;
  ++col;
  if (format == 22) {
    name = intern(p, lim, c->str[MDI_STR_NAME]);
    if (!tab(p)) return false;
    ++col;
    rank = intern(p, lim, c->str[MDI_STR_RANK]);
    if (!tab(p)) return false;
    ++col;
  } else {  // the 20-column table has no name / rank: every row interns ""
    name = c->str[MDI_STR_NAME].add(std::string_view());
    rank = c->str[MDI_STR_RANK].add(std::string_view());
  }
  if (!parse_int(p, lim, &nal) || !tab(p)) return false;
  ++col;
  const int32_t strand = intern(p, lim, c->str[MDI_STR_STRAND]);
  if (!tab(p)) return false;
  ++col;
  if (!parse_int(p, lim, &pos)) return false;
  ++col;
  for (int j = 0; j < 16; ++j) {  // column-major: counts[j][rows]
    int64_t v;
    if (!tab(p) || !parse_int(p, lim, &v)) return false;
    o.counts[(int64_t)j * o.rows + r] = v;
    ++col;
  }
  while (*p == '\r') ++p;
  if (*p != '\n') return false;
  ++p;
  o.tax_id[r] = tid;
  o.nal[r] = nal;
  o.pos[r] = pos;
  o.code[MDI_STR_NAME][r] = name;
  o.code[MDI_STR_RANK][r] = rank;
  o.code[MDI_STR_STRAND][r] = strand;
  return true;
}

void parse_chunk(Chunk* c, int format, const Out& o) {
  const char* p = c->begin;
  const char* end = c->end;
  int64_t r = c->row0;
  const int64_t rend = c->row0 + c->rows;
  // a last line without its newline: parsed from a copy that has one (its
  // string fields then view the copy, which lives as long as the chunk)
  const char* tail = end;
  size_t tail_len = 0;
  if (end > p && end[-1] != '\n') {
    const char* q = end;
    while (q > p && q[-1] != '\n') --q;
    tail = q;
    c->tail.assign(q, (size_t)(end - q));
    c->tail.push_back('\n');
    tail_len = c->tail.size();
    c->tail.append(8, '\0');  // readable padding for parse_int's 8-byte loads
  }
  int col = 0;
  auto bad = [&](int colno) {
    c->err = MDI_E_PARSE;
    c->bad_row = r - c->row0;
    c->bad_col = colno;
  };
  for (int part = 0; part < 2; ++part) {
    const char* q = part == 0 ? p : c->tail.data();
    const char* qe = part == 0 ? tail : c->tail.data() + tail_len;
    const char* lim = part == 0 ? o.map_end : c->tail.data() + c->tail.size();
    while (q < qe) {
      if (*q == '\n' || *q == '\r') {  // blank line
        ++q;
        continue;
      }
      if (r >= rend) return bad(0);  // (rows were counted on the same bytes)
      if (!parse_line(q, lim, format, o, c, r, col)) return bad(col);
      ++r;
    }
    if (c->tail.empty()) break;
  }
}

template <typename F>
void parallel_chunks(std::vector<Chunk>& chunks, F f) {
  std::vector<std::thread> pool;
  for (size_t i = 1; i < chunks.size(); ++i) pool.emplace_back(f, i);
  if (!chunks.empty()) f((size_t)0);
  for (auto& th : pool) th.join();
}

}  // namespace

// The release worker of mdi_free: one thread, started on the first deferred
// release, fed through a queue, drained and joined when the library unloads
// (static destructor: exit(), or dlclose of the last handle).
static void release_table(mdi_table* x) {
  if (x->map && x->map != MAP_FAILED) munmap(x->map, x->size);
  delete x;
}

namespace {
struct ReleaseWorker {
  std::mutex mu;
  std::condition_variable cv;
  std::deque<mdi_table*> q;
  std::thread th;
  bool stop = false;

  void push(mdi_table* t) {
    {
      std::lock_guard<std::mutex> g(mu);
      q.push_back(t);
      if (!th.joinable()) th = std::thread([this] { run(); });
    }
    cv.notify_one();
  }
  void run() {
    std::unique_lock<std::mutex> g(mu);
    while (true) {
      cv.wait(g, [this] { return stop || !q.empty(); });
      if (q.empty()) return;  // (stop, and nothing left)
      mdi_table* t = q.front();
      q.pop_front();
      g.unlock();
      release_table(t);
      g.lock();
    }
  }
  ~ReleaseWorker() {
    {
      std::lock_guard<std::mutex> g(mu);
      stop = true;
    }
    cv.notify_one();
    if (th.joinable()) th.join();
  }
};
ReleaseWorker g_release;
}  // namespace

extern "C" {

int mdi_default_threads(void) {
  if (const char* e = std::getenv("OMP_NUM_THREADS")) {
    const int v = std::atoi(e);
    if (v > 0) return v;
  }
  cpu_set_t set;
  CPU_ZERO(&set);
  if (sched_getaffinity(0, sizeof(set), &set) == 0) {
    const int c = CPU_COUNT(&set);
    if (c > 0) return c;
  }
  const int h = (int)std::thread::hardware_concurrency();
  return h > 0 ? h : 1;
}

int mdi_open(const char* path, int n_threads, mdi_table** out) {
  if (!path || !out) return fail(MDI_E_ARG, "null argument");
  *out = nullptr;
  const int fd = open(path, O_RDONLY);
  if (fd < 0) return fail(MDI_E_IO, "cannot open file");
  struct stat sb;
  if (fstat(fd, &sb) != 0) {
    close(fd);
    return fail(MDI_E_IO, "cannot stat file");
  }
  mdi_table* t = new mdi_table();
  t->size = (size_t)sb.st_size;
  if (t->size > 0) {
    // (no MAP_POPULATE: the row count below faults the pages in on every
    // thread at once -- populating them here took ~13 ms on one thread)
    static const bool populate = [] {
      const char* e = std::getenv("MDI_POPULATE");
      return e != nullptr && std::atoi(e) != 0;
    }();
    t->map = mmap(nullptr, t->size, PROT_READ, MAP_PRIVATE | (populate ? MAP_POPULATE : 0), fd, 0);
    if (t->map == MAP_FAILED) {
      close(fd);
      delete t;
      return fail(MDI_E_IO, "mmap failed");
    }
  }
  close(fd);
  const char* base = (const char*)t->map;
  const char* p = base;
  const char* end = base + t->size;
  // format: a '#' header line or 20 tab-separated fields -> the data/input table
  if (t->size > 0) {
    const char* eol = (const char*)memchr(p, '\n', t->size);
    const char* le = eol ? eol : end;
    int tabs = 0;
    for (const char* q = p; q < le; ++q) tabs += *q == '\t';
    if (*p == '#' || tabs + 1 == 20) t->format = 20;
    if (*p == '#') {
      p = eol ? eol + 1 : end;
      t->first_line = 2;
    }
  }
  t->data = p;
  int nt = n_threads > 0 ? n_threads : mdi_default_threads();
  if (nt < 1) nt = 1;
  const size_t span = (size_t)(end - p);
  if (span < ((size_t)1 << 20)) nt = 1;
  std::vector<const char*> cuts{p};
  for (int i = 1; i < nt; ++i) {
    const char* q = p + span * i / nt;
    if (q <= cuts.back()) continue;
    const char* nl = (const char*)memchr(q, '\n', (size_t)(end - q));
    q = nl ? nl + 1 : end;
    if (q > cuts.back() && q < end) cuts.push_back(q);
  }
  cuts.push_back(end);
  t->chunks.resize(cuts.size() - 1);
  for (size_t i = 0; i < t->chunks.size(); ++i) {
    t->chunks[i].begin = cuts[i];
    t->chunks[i].end = cuts[i + 1];
  }
  parallel_chunks(t->chunks, [&](size_t i) { t->chunks[i].rows = count_rows(t->chunks[i].begin, t->chunks[i].end); });
  int64_t r = 0;
  for (Chunk& c : t->chunks) {
    c.row0 = r;
    r += c.rows;
  }
  t->rows = r;
  *out = t;
  g_err[0] = '\0';
  return 0;
}

int mdi_format(const mdi_table* t) { return t ? t->format : MDI_E_ARG; }
int64_t mdi_rows(const mdi_table* t) { return t ? t->rows : MDI_E_ARG; }

int mdi_parse_into(mdi_table* t, int64_t* tax_id, int64_t* n_alignments, int64_t* position, int64_t* counts16,
                   int32_t* name_code, int32_t* rank_code, int32_t* strand_code) {
  if (!t || !tax_id || !n_alignments || !position || !counts16 || !name_code || !rank_code || !strand_code)
    return fail(MDI_E_ARG, "null argument");
  if (t->parsed) return fail(MDI_E_ARG, "table already parsed");
  const Out o{tax_id, n_alignments, position, counts16, {name_code, rank_code, strand_code}, t->rows,
              (const char*)t->map + t->size};
  const int format = t->format;
  parallel_chunks(t->chunks, [&](size_t i) { parse_chunk(&t->chunks[i], format, o); });
  for (const Chunk& c : t->chunks)
    if (c.err) {  // line number of the malformed row: count lines before its chunk
      long line = t->first_line;
      for (const char* q = t->data; q < c.begin;) {
        const char* nl = (const char*)memchr(q, '\n', (size_t)(c.begin - q));
        if (!nl) break;
        ++line;
        q = nl + 1;
      }
      return fail(MDI_E_PARSE, "line %ld, column %ld: malformed value", line + c.bad_row, (long)c.bad_col + 1);
    }
  // merge the chunks' string tables (file order) and rewrite the codes
  int32_t* codes[3] = {name_code, rank_code, strand_code};
  for (int w = 0; w < 3; ++w) {
    std::unordered_map<std::string_view, int32_t> ids;
    std::vector<std::vector<int32_t>> remap(t->chunks.size());
    for (size_t i = 0; i < t->chunks.size(); ++i) {
      const LocalStrings& ls = t->chunks[i].str[w];
      remap[i].resize(ls.uniq.size());
      for (size_t k = 0; k < ls.uniq.size(); ++k) {
        auto it = ids.find(ls.uniq[k]);
        if (it == ids.end()) {
          const int32_t id = (int32_t)t->strings[w].size();
          t->strings[w].emplace_back(ls.uniq[k]);
          ids.emplace(ls.uniq[k], id);  // keys view the mapping, alive until mdi_free
          remap[i][k] = id;
        } else {
          remap[i][k] = it->second;
        }
      }
    }
    parallel_chunks(t->chunks, [&](size_t i) {
      int32_t* c = codes[w] + t->chunks[i].row0;
      const std::vector<int32_t>& m = remap[i];
      for (int64_t k = 0; k < t->chunks[i].rows; ++k) c[k] = m[(size_t)c[k]];
    });
  }
  t->parsed = true;
  g_err[0] = '\0';
  return 0;
}

int64_t mdi_n_strings(const mdi_table* t, int which) {
  if (!t || which < 0 || which > 2) return MDI_E_ARG;
  return (int64_t)t->strings[which].size();
}

int64_t mdi_string_bytes(const mdi_table* t, int which) {
  if (!t || which < 0 || which > 2) return MDI_E_ARG;
  int64_t b = 0;
  for (const std::string& s : t->strings[which]) b += (int64_t)s.size();
  return b;
}

int mdi_strings(const mdi_table* t, int which, char* buf, int64_t* offsets) {
  if (!t || which < 0 || which > 2 || !buf || !offsets) return fail(MDI_E_ARG, "bad arguments");
  int64_t o = 0;
  size_t i = 0;
  for (const std::string& s : t->strings[which]) {
    offsets[i++] = o;
    std::memcpy(buf + o, s.data(), s.size());
    o += (int64_t)s.size();
  }
  offsets[i] = o;
  return 0;
}

void mdi_free(mdi_table* t) {
  if (!t) return;
  // unmapping a populated 300 MB mapping takes ~20 ms of page-table teardown,
  // and the chunks' string tables (~1e5 hash nodes and strings per file) ~8 ms
  // of frees: both off the caller's thread (nothing views the mapping or the
  // tables any more: the caller copied the strings out with mdi_strings), on
  // the library's release worker, which the library's destructor drains and
  // joins -- a process that exits right after its last mdi_free does not race
  // the allocator's teardown
  if (t->size >= ((size_t)1 << 24)) g_release.push(t);
  else release_table(t);
}

const char* mdi_last_error(void) { return g_err; }

}  // extern "C"
