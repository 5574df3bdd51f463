// codec.h — host I/O of the prover boundary: CBOR Vec<BlockSummary> decode
// (crates/sezkp-core/src/io.rs:57-65), ProofArtifact CBOR encode (io.rs:176-183,
// artifact.rs:55-68), bincode 1.3.3 fixint-LE primitives (proof.rs:80-98) and
// the manifest commitment (crates/sezkp-merkle/src/lib.rs:85-157).
#pragma once
#include <stdint.h>

#include <string>
#include <vector>

#include "../../include/sezkp_stark.h"

namespace sezkp {

// Owned struct-of-arrays storage behind a sezkp_block_view.
struct BlockStore {
  uint32_t tau = 0;
  std::vector<uint16_t> version, ctrl_in, ctrl_out;
  std::vector<uint32_t> block_id, off_in, off_out;
  std::vector<uint64_t> step_lo, step_hi, step_start;
  std::vector<int64_t> in_head_in, in_head_out, win_left, win_right;
  std::vector<int8_t> input_mv, mv;
  std::vector<uint8_t> has_write;
  std::vector<uint16_t> wsym;
  sezkp_block_view view{};
  void bind();  // (re)point view at the vectors
};
bool decode_blocks_cbor(const uint8_t* data, size_t len, BlockStore& out, std::string& err);
bool decode_blocks_json(const char* data, size_t len, BlockStore& out, std::string& err);
bool decode_blocks_jsonl(const char* data, size_t len, BlockStore& out, std::string& err);
// sliced ingest: the lines starting in the byte range [lo, hi) (cut at line
// ends): block fields + step counts (steps = false: the step arrays stay
// empty) or the full blocks; line_off = each line's byte offset
bool decode_blocks_jsonl_meta(const char* data, size_t len, size_t lo, size_t hi, BlockStore& out,
                              std::vector<uint64_t>& line_off, std::string& err, bool steps = false);
std::string encode_blocks_jsonl(const sezkp_block_view& v);
std::vector<uint8_t> encode_blocks_cbor(const sezkp_block_view& v);
// partition_trace (partition.rs:43-150) of a step-major movement log into blocks of b steps
void partition_trace(BlockStore& s, uint64_t t, uint32_t tau, uint32_t b, const int8_t* input_mv, const int8_t* mv,
                     const uint8_t* has_write, const uint16_t* wsym);
bool decode_manifest_cbor(const uint8_t* data, size_t len, uint8_t root[32], uint32_t* n_leaves, std::string& err);
bool decode_manifest_json(const char* data, size_t len, uint8_t root[32], uint32_t* n_leaves, std::string& err);

struct Artifact {
  std::string backend;
  std::vector<uint8_t> manifest_root;
  std::vector<uint8_t> proof_bytes;
  std::string meta_json;
};
bool decode_artifact_cbor(const uint8_t* data, size_t len, Artifact& out, std::string& err);

// ciborium-compatible encoding of ProofArtifact with meta keys in sorted order.
struct MetaEntry {
  std::string key;
  bool is_str;
  std::string s;
  uint64_t u;
};
std::vector<uint8_t> encode_artifact_cbor(const std::string& backend, const uint8_t manifest_root[32],
                                          const std::vector<uint8_t>& proof, std::vector<MetaEntry> meta);
std::string meta_to_json(std::vector<MetaEntry> meta);
std::vector<uint8_t> encode_manifest_cbor(const uint8_t root[32], uint32_t n_leaves);

// bincode 1.3.3 (default options: fixint, little endian)
struct BinWriter {
  std::vector<uint8_t> b;
  void u64(uint64_t x) {
    for (int i = 0; i < 8; i++) b.push_back((uint8_t)(x >> (8 * i)));
  }
  void raw(const void* p, size_t n) {
    const uint8_t* q = static_cast<const uint8_t*>(p);
    b.insert(b.end(), q, q + n);
  }
};

void manifest_leaf_hash(const sezkp_block_view& v, uint32_t k, uint8_t out[32]);
void manifest_root(const sezkp_block_view& v, uint8_t out[32]);
// Frontier root of the .jsonl commit path (lib.rs:167-208, 259-330)
void manifest_frontier_root(const sezkp_block_view& v, uint8_t out[32]);
// the same two roots over given leaf hashes (distributed precheck)
void merkle_root_of_leaves(const uint8_t* leaves, size_t n, bool frontier, uint8_t out[32]);
void frontier_root_of_leaves(const uint8_t* leaves, size_t n, uint8_t out[32]);

}  // namespace sezkp
