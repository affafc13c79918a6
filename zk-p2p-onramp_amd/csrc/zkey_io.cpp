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
#include <cstdio>
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

std::vector<uint8_t> gunzip_if_needed(std::vector<uint8_t> in) {
  if (in.size() < 2 || in[0] != 0x1f || in[1] != 0x8b) return in;
  std::vector<uint8_t> out;
  out.reserve(in.size() * 3);
  z_stream zs;
  std::memset(&zs, 0, sizeof zs);
  if (inflateInit2(&zs, 16 + MAX_WBITS) != Z_OK) throw ZkpError(ZKP_ERR_INTERNAL, "zlib init failed");
  const size_t CH = size_t(1) << 24;
  size_t fed = 0;  // input bytes handed to zlib so far
  auto refill = [&] {
    const size_t n = std::min<size_t>(in.size() - fed, size_t(1) << 30);
    zs.next_in = in.data() + fed;
    zs.avail_in = (uInt)n;
    fed += n;
  };
  refill();
  for (;;) {
    const size_t at = out.size();
    out.resize(at + CH);
    zs.next_out = out.data() + at;
    zs.avail_out = (uInt)CH;
    const int rc = inflate(&zs, Z_NO_FLUSH);
    out.resize(at + (CH - zs.avail_out));
    if (rc == Z_STREAM_END) {
      const size_t used = fed - zs.avail_in;  // input consumed so far
      if (used + 2 <= in.size() && in[used] == 0x1f && in[used + 1] == 0x8b) {  // next gzip member
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
      if (fed == in.size() && zs.avail_out != 0) {
        inflateEnd(&zs);
        throw ZkpError(ZKP_ERR_FORMAT, "zkey: truncated gzip data");
      }
      if (fed < in.size()) refill();
    }
  }
  inflateEnd(&zs);
  return out;
}

// true when buf is exactly one binfile with magic `magic` (section walk ends at the end)
static bool whole_binfile(const std::vector<uint8_t>& buf, const char* magic) {
  if (buf.size() < 12 || std::memcmp(buf.data(), magic, 4) != 0) return false;
  uint32_t nsec;
  std::memcpy(&nsec, buf.data() + 8, 4);
  size_t pos = 12;
  for (uint32_t i = 0; i < nsec; ++i) {
    if (pos + 12 > buf.size()) return false;
    uint64_t sl;
    std::memcpy(&sl, buf.data() + pos + 4, 8);
    pos += 12;
    if (sl > buf.size() - pos) return false;
    pos += sl;
  }
  return pos == buf.size();
}

std::vector<uint8_t> merge_zkey_chunks(std::vector<std::vector<uint8_t>> chunks) {
  if (chunks.empty()) throw ZkpError(ZKP_ERR_INVALID_ARG, "no zkey chunks");
  for (auto& c : chunks) c = gunzip_if_needed(std::move(c));
  if (chunks.size() == 1) return std::move(chunks[0]);
  // byte split?
  size_t total = 0;
  for (auto& c : chunks) total += c.size();
  if (chunks[0].size() >= 4 && std::memcmp(chunks[0].data(), "zkey", 4) == 0) {
    std::vector<uint8_t> cat;
    cat.reserve(total);
    for (auto& c : chunks) cat.insert(cat.end(), c.begin(), c.end());
    if (whole_binfile(cat, "zkey")) return cat;
  }
  // section split: merge the sections of per-chunk binfiles
  uint32_t version = 0;
  std::map<uint32_t, std::pair<const uint8_t*, uint64_t>> secs;
  for (size_t k = 0; k < chunks.size(); ++k) {
    const auto& c = chunks[k];
    if (!whole_binfile(c, "zkey"))
      throw ZkpError(ZKP_ERR_FORMAT, "zkey chunk " + std::to_string(k) + ": Invalid File format");
    uint32_t v, nsec;
    std::memcpy(&v, c.data() + 4, 4);
    std::memcpy(&nsec, c.data() + 8, 4);
    if (k && v != version) throw ZkpError(ZKP_ERR_FORMAT, "zkey chunks: version mismatch");
    version = v;
    size_t pos = 12;
    for (uint32_t i = 0; i < nsec; ++i) {
      uint32_t id;
      uint64_t sl;
      std::memcpy(&id, c.data() + pos, 4);
      std::memcpy(&sl, c.data() + pos + 4, 8);
      pos += 12;
      if (!secs.emplace(id, std::make_pair(c.data() + pos, sl)).second)
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
  for (auto& [id, s] : secs) {
    put(&id, 4);
    put(&s.second, 8);
    put(s.first, s.second);
  }
  return out;
}

std::vector<uint8_t> read_zkey_source(const std::string& path) {
  if (file_exists(path)) return gunzip_if_needed(read_raw(path));
  if (file_exists(path + ".gz")) return gunzip_if_needed(read_raw(path + ".gz"));
  // chunks path{a..z}[.gz], in suffix order (the app uses b..k)
  std::vector<std::vector<uint8_t>> chunks;
  for (char s = 'a'; s <= 'z'; ++s) {
    const std::string p = path + s;
    if (file_exists(p))
      chunks.push_back(read_raw(p));
    else if (file_exists(p + ".gz"))
      chunks.push_back(read_raw(p + ".gz"));
  }
  if (chunks.empty()) throw ZkpError(ZKP_ERR_IO, "cannot open " + path + " (nor .gz, nor chunks " + path + "{a..z})");
  return merge_zkey_chunks(std::move(chunks));
}

std::vector<uint8_t> read_zkey_chunks(const std::vector<std::string>& paths) {
  std::vector<std::vector<uint8_t>> chunks;
  for (auto& p : paths) chunks.push_back(read_raw(p));
  return merge_zkey_chunks(std::move(chunks));
}

}  // namespace zkp
