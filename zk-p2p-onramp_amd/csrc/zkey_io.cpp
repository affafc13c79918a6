// zkey ingestion from files: plain, gzip-compressed, or chunked.
//
// The ZKP2P app ships the proving key as chunks `circuit.zkey{b..k}.gz` (reference
// app/src/helpers/zkp.ts:11-13 zkeySuffix / zkeyExtension, :51-68 download +
// uncompress; circuit/server-scripts/upload_chunked_keys_to_s3.sh:13-22 uploads
// circuit.zkeyb .. circuit.zkeyk) that the browser snarkjs fork reads back as
// `circuit.zkey`.  The chunk layout is that of an un-vendored snarkjs fork
// (dizkus-scripts/3_gen_both_zkeys.sh: vb7401/snarkjs#24981feb), so both plausible
// layouts are accepted and told apart by content:
//   * byte split: the chunks concatenate to one binfile (the first starts with "zkey"
//     and the section walk of the concatenation ends exactly at its end);
//   * section split: every chunk is itself a "zkey" binfile holding some of the
//     sections; they are merged (each section id at most once).
// Each chunk (or the single file) may be gzip-compressed (detected by magic 1f 8b).
#include "zkey_io.hpp"

#include <zlib.h>

#include <algorithm>
#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <exception>
#include <mutex>
#include <thread>
#include <cstring>
#include <fstream>
#include <map>
#include <sys/stat.h>

#include "prover.hpp"

namespace zkp {

static bool file_exists(const std::string& p) {
  struct stat st;
  return ::stat(p.c_str(), &st) == 0 && S_ISREG(st.st_mode);
}

static std::vector<uint8_t> read_raw(const std::string& path) {
  std::ifstream f(path, std::ios::binary | std::ios::ate);
  if (!f) throw ZkpError(ZKP_ERR_IO, "cannot open " + path);
  const std::streamsize n = f.tellg();
  f.seekg(0);
  std::vector<uint8_t> buf((size_t)n);
  if (n && !f.read(reinterpret_cast<char*>(buf.data()), n)) throw ZkpError(ZKP_ERR_IO, "cannot read " + path);
  return buf;
}

// inflate the gzip stream(s) in[0, n) (multi-member ok); appends to `out` when dst == nullptr,
// else writes into [dst, dst + cap) and returns the byte count (cap exceeded: returns cap + 1)
static size_t inflate_gz(const uint8_t* in, size_t n, std::vector<uint8_t>* out, uint8_t* dst, size_t cap) {
  z_stream zs;
  std::memset(&zs, 0, sizeof zs);
  if (inflateInit2(&zs, 16 + MAX_WBITS) != Z_OK) throw ZkpError(ZKP_ERR_INTERNAL, "zlib init failed");
  const size_t CH = size_t(1) << 24;
  size_t fed = 0, written = 0;  // input bytes handed to zlib / output bytes produced
  auto refill = [&] {
    const size_t k = std::min<size_t>(n - fed, size_t(1) << 30);
    zs.next_in = const_cast<uint8_t*>(in) + fed;
    zs.avail_in = (uInt)k;
    fed += k;
  };
  refill();
  for (;;) {
    size_t room;
    if (dst) {
      room = std::min(CH, cap - written);
      if (room == 0) {  // the stream holds more than cap bytes
        inflateEnd(&zs);
        return cap + 1;
      }
      zs.next_out = dst + written;
    } else {
      out->resize(written + CH);
      room = CH;
      zs.next_out = out->data() + written;
    }
    zs.avail_out = (uInt)room;
    const int rc = inflate(&zs, Z_NO_FLUSH);
    written += room - zs.avail_out;
    if (!dst) out->resize(written);
    if (rc == Z_STREAM_END) {
      const size_t used = fed - zs.avail_in;  // input consumed so far
      if (used + 2 <= n && in[used] == 0x1f && in[used + 1] == 0x8b) {  // next gzip member
        inflateReset(&zs);
        fed = used;
        refill();
        continue;
      }
      break;
    }
    if (rc != Z_OK && rc != Z_BUF_ERROR) {
      inflateEnd(&zs);
      throw ZkpError(ZKP_ERR_FORMAT, "zkey: corrupt gzip data");
    }
    if (zs.avail_in == 0) {
      if (fed == n && zs.avail_out != 0) {
        inflateEnd(&zs);
        throw ZkpError(ZKP_ERR_FORMAT, "zkey: truncated gzip data");
      }
      if (fed < n) refill();
    }
  }
  inflateEnd(&zs);
  return written;
}

static bool is_gz(const std::vector<uint8_t>& b) { return b.size() >= 18 && b[0] == 0x1f && b[1] == 0x8b; }

std::vector<uint8_t> gunzip_if_needed(std::vector<uint8_t> in) {
  if (in.size() < 2 || in[0] != 0x1f || in[1] != 0x8b) return in;
  std::vector<uint8_t> out;
  out.reserve(in.size() * 3);
  inflate_gz(in.data(), in.size(), &out, nullptr, 0);
  return out;
}

// run f(k) for k < n on up to hardware_concurrency threads; the first exception is rethrown
template <class Fn>
static void parallel_for(size_t n, Fn f) {
  size_t T = std::max<size_t>(1, std::min<size_t>(n, std::thread::hardware_concurrency()));
  std::atomic<size_t> next{0};
  std::exception_ptr err;
  std::mutex mu;
  std::vector<std::thread> th;
  for (size_t t = 0; t < T; ++t)
    th.emplace_back([&] {
      for (size_t k; (k = next.fetch_add(1)) < n;) {
        try {
          f(k);
        } catch (...) {
          std::lock_guard<std::mutex> g(mu);
          if (!err) err = std::current_exception();
        }
      }
    });
  for (auto& x : th) x.join();
  if (err) std::rethrow_exception(err);
}

// true when buf is exactly one binfile with magic `magic` (section walk ends at the end)
static bool whole_binfile(const uint8_t* buf, size_t size, const char* magic) {
  if (size < 12 || std::memcmp(buf, magic, 4) != 0) return false;
  uint32_t nsec;
  std::memcpy(&nsec, buf + 8, 4);
  size_t pos = 12;
  for (uint32_t i = 0; i < nsec; ++i) {
    if (pos + 12 > size) return false;
    uint64_t sl;
    std::memcpy(&sl, buf + pos + 4, 8);
    pos += 12;
    if (sl > size - pos) return false;
    pos += sl;
  }
  return pos == size;
}

// section split: merge the sections of per-chunk binfiles (views into the chunk bytes)
static std::vector<uint8_t> merge_sections(const std::vector<std::pair<const uint8_t*, size_t>>& chunks) {
  uint32_t version = 0;
  size_t total = 0;
  std::map<uint32_t, std::pair<const uint8_t*, uint64_t>> secs;
  for (size_t k = 0; k < chunks.size(); ++k) {
    const uint8_t* c = chunks[k].first;
    const size_t len = chunks[k].second;
    total += len;
    if (!whole_binfile(c, len, "zkey"))
      throw ZkpError(ZKP_ERR_FORMAT, "zkey chunk " + std::to_string(k) + ": Invalid File format");
    uint32_t v, nsec;
    std::memcpy(&v, c + 4, 4);
    std::memcpy(&nsec, c + 8, 4);
    if (k && v != version) throw ZkpError(ZKP_ERR_FORMAT, "zkey chunks: version mismatch");
    version = v;
    size_t pos = 12;
    for (uint32_t i = 0; i < nsec; ++i) {
      uint32_t id;
      uint64_t sl;
      std::memcpy(&id, c + pos, 4);
      std::memcpy(&sl, c + pos + 4, 8);
      pos += 12;
      if (!secs.emplace(id, std::make_pair(c + pos, sl)).second)
        throw ZkpError(ZKP_ERR_FORMAT, "zkey chunks: section " + std::to_string(id) + " appears twice");
      pos += sl;
    }
  }
  std::vector<uint8_t> out;
  out.reserve(total);
  auto put = [&](const void* p, size_t n) {
    const uint8_t* b = static_cast<const uint8_t*>(p);
    out.insert(out.end(), b, b + n);
  };
  const uint32_t nsec = (uint32_t)secs.size();
  put("zkey", 4);
  put(&version, 4);
  put(&nsec, 4);
  for (auto& [id, sec] : secs) {
    put(&id, 4);
    put(&sec.second, 8);
    put(sec.first, sec.second);
  }
  return out;
}

std::vector<uint8_t> merge_zkey_chunks(std::vector<std::vector<uint8_t>> chunks) {
  if (chunks.empty()) throw ZkpError(ZKP_ERR_INVALID_ARG, "no zkey chunks");
  const size_t K = chunks.size();
  // Cold start (the app's circuit.zkey{b..k}.gz): every chunk inflated in parallel straight into
  // its slot of ONE output buffer, sized from the gzip trailers (ISIZE = length mod 2^32 of the
  // last member); a chunk whose inflated length differs (several members, >= 4 GiB) falls back
  // to inflating into a buffer of its own.
  std::vector<size_t> len(K), off(K + 1, 0);
  for (size_t k = 0; k < K; ++k) {
    const auto& c = chunks[k];
    if (is_gz(c)) {
      uint32_t isz;
      std::memcpy(&isz, c.data() + c.size() - 4, 4);
      len[k] = isz;
    } else {
      len[k] = c.size();
    }
    off[k + 1] = off[k] + len[k];
  }
  std::vector<uint8_t> out(off[K]);
  std::vector<std::vector<uint8_t>> own(K);  // chunks that did not fit their trailer size
  std::vector<char> fits(K, 1);
  parallel_for(K, [&](size_t k) {
    auto& c = chunks[k];
    if (!is_gz(c)) {
      std::memcpy(out.data() + off[k], c.data(), c.size());
    } else {
      const size_t w = inflate_gz(c.data(), c.size(), nullptr, out.data() + off[k], len[k]);
      if (w != len[k]) {
        fits[k] = 0;
        inflate_gz(c.data(), c.size(), &own[k], nullptr, 0);
      }
    }
    std::vector<uint8_t>().swap(c);  // compressed bytes no longer needed
  });
  const bool all_fit = std::all_of(fits.begin(), fits.end(), [](char f) { return f != 0; });
  if (all_fit && (K == 1 || whole_binfile(out.data(), out.size(), "zkey"))) return out;  // single / byte split
  if (K == 1) return std::move(own[0]);
  std::vector<std::pair<const uint8_t*, size_t>> views(K);
  for (size_t k = 0; k < K; ++k)
    views[k] = fits[k] ? std::make_pair((const uint8_t*)out.data() + off[k], len[k])
                       : std::make_pair((const uint8_t*)own[k].data(), own[k].size());
  if (!all_fit) {  // byte split with a multi-member chunk: concatenate the views
    std::vector<uint8_t> cat;
    size_t total = 0;
    for (auto& v : views) total += v.second;
    if (views[0].second >= 4 && std::memcmp(views[0].first, "zkey", 4) == 0) {
      cat.reserve(total);
      for (auto& v : views) cat.insert(cat.end(), v.first, v.first + v.second);
      if (whole_binfile(cat.data(), cat.size(), "zkey")) return cat;
    }
  }
  return merge_sections(views);
}

std::vector<uint8_t> read_zkey_source(const std::string& path) {
  if (file_exists(path)) return gunzip_if_needed(read_raw(path));
  if (file_exists(path + ".gz")) return gunzip_if_needed(read_raw(path + ".gz"));
  // chunks path{a..z}[.gz], in suffix order (the app uses b..k)
  std::vector<std::string> paths;
  for (char s = 'a'; s <= 'z'; ++s) {
    const std::string p = path + s;
    if (file_exists(p))
      paths.push_back(p);
    else if (file_exists(p + ".gz"))
      paths.push_back(p + ".gz");
  }
  if (paths.empty()) throw ZkpError(ZKP_ERR_IO, "cannot open " + path + " (nor .gz, nor chunks " + path + "{a..z})");
  return read_zkey_chunks(paths);
}

std::vector<uint8_t> read_zkey_chunks(const std::vector<std::string>& paths) {
  std::vector<std::vector<uint8_t>> chunks(paths.size());
  parallel_for(paths.size(), [&](size_t k) { chunks[k] = read_raw(paths[k]); });
  return merge_zkey_chunks(std::move(chunks));
}

}  // namespace zkp
