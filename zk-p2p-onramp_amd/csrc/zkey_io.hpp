// zkey ingestion from files: plain, gzip-compressed, or chunked (see zkey_io.cpp).
#pragma once
#include <cstdint>
#include <string>
#include <vector>

namespace zkp {

// inflate a gzip stream (magic 1f 8b, multi-member ok); other bytes pass through
std::vector<uint8_t> gunzip_if_needed(std::vector<uint8_t> in);
// one zkey from chunks (each maybe gzip): byte split or section split
std::vector<uint8_t> merge_zkey_chunks(std::vector<std::vector<uint8_t>> chunks);
// `path` if it exists (maybe gzip), else path.gz, else the chunks path{a..z}[.gz]
std::vector<uint8_t> read_zkey_source(const std::string& path);
// explicit chunk list, in order
std::vector<uint8_t> read_zkey_chunks(const std::vector<std::string>& paths);

}  // namespace zkp
