// cli.cpp — `sezkp-cli` drop-in for the STARK path on MI355X:
//   prove  --backend stark --blocks B --manifest M --out P [--stream] [--assume-committed]
//   verify --backend stark --blocks B --manifest M --proof P [--assume-committed]
//   commit --blocks B(.cbor|.json|.jsonl|.ndjson) --out M
//   verify-commit --blocks B --manifest M
//   export-jsonl --input B(.cbor|.json|.jsonl|.ndjson) --output B.jsonl
// Semantics follow crates/sezkp-cli/src/main.rs:429-578 (manifest precheck,
// .json/.cbor block files only for prove/verify, write_proof_auto by extension)
// and crates/sezkp-merkle/src/lib.rs:259-337 (commit / precheck).
#include <stdio.h>
#include <string.h>

#include <sys/stat.h>

#include <algorithm>
#include <fstream>
#include <sstream>
#include <string>
#include <vector>

#include "../../include/sezkp_stark.h"
#include "codec.h"
#include "host_crypto.h"

using namespace sezkp;

namespace {

std::string ext_lower(const std::string& p) {
  size_t d = p.find_last_of('.');
  size_t s = p.find_last_of('/');
  if (d == std::string::npos || (s != std::string::npos && d < s)) return "";
  std::string e = p.substr(d + 1);
  for (auto& c : e) c = (char)tolower((unsigned char)c);
  return e;
}
std::string hex(const uint8_t* p, size_t n) {
  static const char* H = "0123456789abcdef";
  std::string s;
  for (size_t i = 0; i < n; i++) { s += H[p[i] >> 4]; s += H[p[i] & 15]; }
  return s;
}
bool read_file(const std::string& path, std::vector<uint8_t>& out, std::string& err) {
  std::ifstream f(path, std::ios::binary);
  if (!f) { err = "open " + path; return false; }
  out.assign(std::istreambuf_iterator<char>(f), std::istreambuf_iterator<char>());
  return true;
}
bool write_file(const std::string& path, const std::vector<uint8_t>& data, std::string& err) {
  std::ofstream f(path, std::ios::binary);
  if (!f) { err = "create " + path; return false; }
  f.write((const char*)data.data(), (std::streamsize)data.size());
  return (bool)f;
}

bool is_jsonl_like(const std::string& path) {  // sezkp-merkle lib.rs:410-412
  const std::string e = ext_lower(path);
  return e == "jsonl" || e == "ndjson";
}
bool load_blocks(const std::string& path, BlockStore& bs, std::string& err) {  // io.rs:78-88
  const std::string e = ext_lower(path);
  std::vector<uint8_t> raw;
  if (e != "json" && e != "cbor") {
    err = e.empty() ? "path has no extension (expected .json or .cbor)"
                    : "unsupported blocks extension: " + e + " (supported: .json, .cbor)";
    return false;
  }
  if (!read_file(path, raw, err)) return false;
  if (e == "cbor") return decode_blocks_cbor(raw.data(), raw.size(), bs, err);
  return decode_blocks_json((const char*)raw.data(), raw.size(), bs, err);
}
bool load_manifest(const std::string& path, uint8_t root[32], uint32_t* n_leaves, std::string& err) {
  const std::string e = ext_lower(path);
  std::vector<uint8_t> raw;
  if (e != "json" && e != "cbor") {
    err = e.empty() ? "path has no extension (expected .json or .cbor)" : "unsupported manifest extension: " + e;
    return false;
  }
  if (!read_file(path, raw, err)) return false;
  if (e == "cbor") return decode_manifest_cbor(raw.data(), raw.size(), root, n_leaves, err);
  return decode_manifest_json((const char*)raw.data(), raw.size(), root, n_leaves, err);
}

// serde_json::to_writer_pretty layout of a ProofArtifact
std::string pretty_artifact(const Artifact& a) {
  std::ostringstream o;
  auto arr = [&](const std::vector<uint8_t>& v) {
    if (v.empty()) { o << "[]"; return; }
    o << "[\n";
    for (size_t i = 0; i < v.size(); i++) o << "    " << (unsigned)v[i] << (i + 1 < v.size() ? ",\n" : "\n");
    o << "  ]";
  };
  o << "{\n  \"backend\": \"" << a.backend << "\",\n  \"manifest_root\": ";
  arr(a.manifest_root);
  o << ",\n  \"proof_bytes\": ";
  arr(a.proof_bytes);
  o << ",\n  \"meta\": " << a.meta_json << "\n}";
  return o.str();
}

struct Args {
  std::string cmd, backend = "stark", blocks, manifest, out, proof, input;
  bool stream = false, assume = false;
  std::string t = "32", b = "4", tau = "2";  // simulate defaults (main.rs:87-100)
};

// The blocks file of `commit` and of the precheck: .jsonl/.ndjson through the
// line reader (io_jsonl.rs:43-84), .json/.cbor through read_block_summaries_auto
bool load_blocks_any(const std::string& path, BlockStore& bs, std::string& err) {
  if (!is_jsonl_like(path)) return load_blocks(path, bs, err);
  std::vector<uint8_t> raw;
  if (!read_file(path, raw, err)) return false;
  return decode_blocks_jsonl((const char*)raw.data(), raw.size(), bs, err);
}
// commit_block_file (lib.rs:259-295): the Frontier root for JSON Lines, the
// batch merkle_root otherwise
void file_root(const std::string& path, const BlockStore& bs, uint8_t root[32]) {
  if (is_jsonl_like(path)) manifest_frontier_root(bs.view, root);
  else manifest_root(bs.view, root);
}

// verify_block_file_against_manifest (lib.rs:302-337), run on the blocks path
// before anything else reads it (main.rs:454-457). `bs` keeps the decoded
// blocks so a .json/.cbor file is read once.
int precheck(const Args& a, BlockStore& bs) {
  uint8_t mroot[32], got[32];
  uint32_t nl = 0;
  std::string err;
  if (!load_manifest(a.manifest, mroot, &nl, err)) {
    fprintf(stderr, "Error: blocks/manifest mismatch: %s\n", err.c_str());
    return 1;
  }
  if (!load_blocks_any(a.blocks, bs, err)) {
    fprintf(stderr, "Error: blocks/manifest mismatch: read blocks %s: %s\n", a.blocks.c_str(), err.c_str());
    return 1;
  }
  file_root(a.blocks, bs, got);
  if (memcmp(got, mroot, 32) != 0) {
    fprintf(stderr, "Error: blocks/manifest mismatch: root mismatch: manifest=%s, recomputed=%s\n",
            hex(mroot, 32).c_str(), hex(got, 32).c_str());
    return 1;
  }
  if (nl != bs.view.n_blocks) {
    fprintf(stderr, "Error: blocks/manifest mismatch: leaf count mismatch: manifest=%u, recomputed=%u\n", nl,
            bs.view.n_blocks);
    return 1;
  }
  return 0;
}

// precheck unless --assume-committed, then the manifest, then the blocks
// through read_block_summaries_auto (.json/.cbor only: a .jsonl file that
// passed the precheck is refused here, as main.rs:503-513 does)
int load_inputs(const Args& a, BlockStore& bs, uint8_t mroot[32]) {
  std::string err;
  bool have = false;
  if (!a.assume) {
    if (precheck(a, bs)) return 1;
    have = !is_jsonl_like(a.blocks);
  }
  if (!load_manifest(a.manifest, mroot, nullptr, err)) { fprintf(stderr, "Error: reading manifest: %s\n", err.c_str()); return 1; }
  if (!have && !load_blocks(a.blocks, bs, err)) { fprintf(stderr, "Error: reading blocks: %s\n", err.c_str()); return 1; }
  return 0;
}

int cmd_prove(const Args& a) {
  std::string err;
  BlockStore bs;
  uint8_t mroot[32];
  if (load_inputs(a, bs, mroot)) return 1;
  sezkp_buf art{};
  char msg[512] = {0};
  const int32_t rc = sezkp_stark_v1_prove_artifact_cbor(&bs.view, mroot, a.stream ? SEZKP_FLAG_STREAMING : 0, &art,
                                                        msg, sizeof msg);
  if (rc) { fprintf(stderr, "Error: stark-v1 proof failed: %s\n", msg); return 1; }
  std::vector<uint8_t> cbor(art.data, art.data + art.len);
  sezkp_buf_free(&art);
  Artifact dec;
  decode_artifact_cbor(cbor.data(), cbor.size(), dec, err);
  std::vector<uint8_t> outb = cbor;
  if (ext_lower(a.out) != "cbor") {  // write_proof_auto: JSON unless .cbor (io.rs:199-205)
    const bool streaming = a.stream;
    uint64_t domain_n = 0;
    for (int i = 7; i >= 0; i--) domain_n = (domain_n << 8) | dec.proof_bytes[i];
    std::vector<MetaEntry> meta = {{"proto", true, "stark-v1", 0}, {"domain_n", false, "", domain_n},
                                   {"tau", false, "", bs.view.tau}};
    if (streaming) meta.push_back({"mode", true, "streaming", 0});
    // serde_json pretty nests the meta object one level deeper
    std::string mj = meta_to_json(meta);
    std::string nested = "{\n";
    {
      std::vector<MetaEntry> m = meta;
      std::sort(m.begin(), m.end(), [](const MetaEntry& x, const MetaEntry& y) { return x.key < y.key; });
      for (size_t i = 0; i < m.size(); i++)
        nested += "    \"" + m[i].key + "\": " + (m[i].is_str ? "\"" + m[i].s + "\"" : std::to_string(m[i].u)) +
                  (i + 1 < m.size() ? ",\n" : "\n");
      nested += "  }";
    }
    (void)mj;
    dec.meta_json = nested;
    std::string js = pretty_artifact(dec);
    outb.assign(js.begin(), js.end());
  }
  if (!write_file(a.out, outb, err)) { fprintf(stderr, "Error: writing proof to %s: %s\n", a.out.c_str(), err.c_str()); return 1; }
  printf("Proved with Stark, wrote %s (%zu bytes)\n", a.out.c_str(), dec.proof_bytes.size());
  return 0;
}

int cmd_verify(const Args& a) {
  std::string err;
  BlockStore bs;
  uint8_t mroot[32];
  if (load_inputs(a, bs, mroot)) return 1;
  std::vector<uint8_t> raw;
  if (!read_file(a.proof, raw, err)) { fprintf(stderr, "Error: reading proof artifact: %s\n", err.c_str()); return 1; }
  if (ext_lower(a.proof) != "cbor") { fprintf(stderr, "Error: only .cbor proof artifacts are supported for verify\n"); return 1; }
  Artifact art;
  if (!decode_artifact_cbor(raw.data(), raw.size(), art, err)) { fprintf(stderr, "Error: %s\n", err.c_str()); return 1; }
  if (art.backend != "stark") { fprintf(stderr, "Error: stark-v1 verification failed: backend kind mismatch: expected STARK\n"); return 1; }
  if (art.manifest_root.size() != 32 || memcmp(art.manifest_root.data(), mroot, 32)) {
    fprintf(stderr, "Error: stark-v1 verification failed: manifest root mismatch\n");
    return 1;
  }
  char msg[512] = {0};
  if (sezkp_stark_v1_verify(art.proof_bytes.data(), art.proof_bytes.size(), &bs.view, mroot, msg, sizeof msg)) {
    fprintf(stderr, "Error: stark-v1 verification failed: %s\n", msg);
    return 1;
  }
  printf("OK: proof verified\n");
  return 0;
}

int cmd_commit(const Args& a) {
  std::string err;
  BlockStore bs;
  if (!load_blocks_any(a.blocks, bs, err)) { fprintf(stderr, "Error: read blocks %s: %s\n", a.blocks.c_str(), err.c_str()); return 1; }
  uint8_t root[32];
  file_root(a.blocks, bs, root);
  std::vector<uint8_t> out;
  if (ext_lower(a.out) == "cbor") out = encode_manifest_cbor(root, bs.view.n_blocks);
  else {
    std::string s = "{\n  \"version\": 1,\n  \"root\": [\n";
    for (int i = 0; i < 32; i++) s += "    " + std::to_string(root[i]) + (i < 31 ? ",\n" : "\n");
    s += "  ],\n  \"n_leaves\": " + std::to_string(bs.view.n_blocks) + "\n}";
    out.assign(s.begin(), s.end());
  }
  if (!write_file(a.out, out, err)) { fprintf(stderr, "Error: %s\n", err.c_str()); return 1; }
  printf("Committed %u leaves, root=%s, wrote manifest %s\n", bs.view.n_blocks, hex(root, 32).c_str(), a.out.c_str());
  return 0;
}

// `verify-commit` (main.rs:377-398): the precheck of prove/verify on its own
int cmd_verify_commit(const Args& a) {
  BlockStore bs;
  if (precheck(a, bs)) return 1;
  printf("OK: %s matches manifest %s\n", a.blocks.c_str(), a.manifest.c_str());
  return 0;
}

// mkdir -p of the output's parent directory (main.rs:299-307)
bool ensure_parent_dir(const std::string& path, std::string& err) {
  const size_t s = path.find_last_of('/');
  if (s == std::string::npos || s == 0) return true;
  const std::string dir = path.substr(0, s);
  for (size_t i = 1; i <= dir.size(); i++) {
    if (i < dir.size() && dir[i] != '/') continue;
    const std::string part = dir.substr(0, i);
    struct stat st;
    if (stat(part.c_str(), &st) == 0) {
      if (!S_ISDIR(st.st_mode)) { err = "creating parent directory " + dir + ": not a directory"; return false; }
    } else if (mkdir(part.c_str(), 0777) != 0) {
      err = "creating parent directory " + dir;
      return false;
    }
  }
  return true;
}

// `export-jsonl` (main.rs:400-424): any blocks file (stream_block_summaries_auto,
// io.rs:111-139: .jsonl/.ndjson, .json, .cbor) -> one serde_json object per line
// (the layout of write_block_summaries_jsonl, io_jsonl.rs:93-106)
int cmd_export_jsonl(const Args& a) {
  if (a.input.empty() || a.out.empty()) { fprintf(stderr, "Error: export-jsonl needs --input and --output\n"); return 2; }
  const std::string e = ext_lower(a.input);
  if (e != "jsonl" && e != "ndjson" && e != "json" && e != "cbor") {
    fprintf(stderr, "Error: open input stream: %s\n",
            e.empty() ? "path has no extension (expected .json, .cbor, .jsonl, or .ndjson)"
                      : ("unsupported blocks extension: " + e + " (supported: .json, .cbor, .jsonl, .ndjson)").c_str());
    return 1;
  }
  std::string err;
  BlockStore bs;
  if (!load_blocks_any(a.input, bs, err)) { fprintf(stderr, "Error: open input stream: %s\n", err.c_str()); return 1; }
  sezkp_buf buf{};
  const int32_t rc = sezkp_blocks_encode_jsonl(&bs.view, &buf);
  if (rc != SEZKP_OK) { fprintf(stderr, "Error: serialize block as JSON line (%d)\n", rc); return 1; }
  std::vector<uint8_t> out(buf.data, buf.data + buf.len);
  sezkp_buf_free(&buf);
  if (!ensure_parent_dir(a.out, err) || !write_file(a.out, out, err)) {
    fprintf(stderr, "Error: %s\n", err.c_str());
    return 1;
  }
  printf("Exported %u blocks \xe2\x86\x92 %s\n", bs.view.n_blocks, a.out.c_str());
  return 0;
}

// `simulate` (main.rs:317-350): generate_trace + partition_trace, written as
// CBOR (.cbor) or NDJSON (.jsonl/.ndjson) by extension
int cmd_simulate(const Args& a) {
  char* end = nullptr;
  const unsigned long long t = strtoull(a.t.c_str(), &end, 10);
  const unsigned long long b = strtoull(a.b.c_str(), nullptr, 10);
  const unsigned long long tau = strtoull(a.tau.c_str(), nullptr, 10);
  if (t == 0 || t > 0xFFFFFFFFull || b == 0 || tau == 0 || tau > 255) {
    fprintf(stderr, "Error: need --t in 1..=2^32-1, --b >= 1, --tau in 1..=255\n");
    return 2;
  }
  if (b > t) {
    fprintf(stderr, "Error: number of blocks b (%llu) cannot exceed trace length T (%llu)\n", b, t);
    return 1;
  }
  const std::string e = ext_lower(a.out);
  if (e != "cbor" && e != "jsonl" && e != "ndjson") {
    fprintf(stderr, "Error: --out-blocks must end in .cbor, .jsonl or .ndjson\n");
    return 2;
  }
  sezkp_blocks* h = nullptr;
  char err[512] = {0};
  if (sezkp_simulate_blocks(t, (uint32_t)b, (uint32_t)tau, 42, &h, err, sizeof err) != SEZKP_OK) {
    fprintf(stderr, "Error: %s\n", err);
    return 1;
  }
  const sezkp_block_view* v = sezkp_blocks_view(h);
  const uint32_t nb = v->n_blocks;
  sezkp_buf buf{};
  const int32_t rc = e == "cbor" ? sezkp_blocks_encode_cbor(v, &buf) : sezkp_blocks_encode_jsonl(v, &buf);
  sezkp_blocks_free(h);
  if (rc != SEZKP_OK) { fprintf(stderr, "Error: encoding blocks failed (%d)\n", rc); return 1; }
  std::vector<uint8_t> out(buf.data, buf.data + buf.len);
  sezkp_buf_free(&buf);
  std::string werr;
  if (!write_file(a.out, out, werr)) { fprintf(stderr, "Error: %s\n", werr.c_str()); return 1; }
  printf("Simulated trace: T=%llu, b=%llu, \xcf\x84=%llu \xe2\x86\x92 %u blocks \xe2\x86\x92 %s\n", t, b, tau, nb,
         a.out.c_str());
  return 0;
}

void usage() {
  fprintf(stderr,
          "usage: sezkp-cli prove  --backend stark --blocks B --manifest M --out P [--stream] [--assume-committed]\n"
          "       sezkp-cli verify --backend stark --blocks B --manifest M --proof P [--assume-committed]\n"
          "       sezkp-cli commit --blocks B --out M\n"
          "       sezkp-cli verify-commit --blocks B --manifest M\n"
          "       sezkp-cli export-jsonl --input B --output B.jsonl\n"
          "       sezkp-cli simulate --t T --b STEPS_PER_BLOCK --tau TAU --out-blocks B(.cbor|.jsonl)\n");
}

}  // namespace

int main(int argc, char** argv) {
  if (argc < 2) { usage(); return 2; }
  Args a;
  a.cmd = argv[1];
  for (int i = 2; i < argc; i++) {
    std::string s = argv[i];
    auto val = [&](std::string& dst) {
      if (i + 1 >= argc) { usage(); exit(2); }
      dst = argv[++i];
    };
    if (s == "--backend" || s == "-b") val(a.backend);
    else if (s == "--blocks") val(a.blocks);
    else if (s == "--manifest") val(a.manifest);
    else if (s == "--out" || s == "-o") val(a.out);
    else if (s == "--proof") val(a.proof);
    else if (s == "--out-blocks" || s == "--output") val(a.out);
    else if (s == "--input") val(a.input);
    else if (s == "--t") val(a.t);
    else if (s == "--b") val(a.b);
    else if (s == "--tau") val(a.tau);
    else if (s == "--stream") a.stream = true;
    else if (s == "--assume-committed") a.assume = true;
    else { fprintf(stderr, "unknown argument %s\n", s.c_str()); usage(); return 2; }
  }
  for (auto& c : a.backend) c = (char)tolower((unsigned char)c);
  if (a.cmd == "commit") return cmd_commit(a);
  if (a.cmd == "simulate") return cmd_simulate(a);
  if (a.cmd == "verify-commit") return cmd_verify_commit(a);
  if (a.cmd == "export-jsonl") return cmd_export_jsonl(a);
  if (a.backend != "stark") {
    fprintf(stderr, "Error: only --backend stark is implemented by the MI355X build\n");
    return 2;
  }
  if (a.cmd == "prove") return cmd_prove(a);
  if (a.cmd == "verify") return cmd_verify(a);
  usage();
  return 2;
}
