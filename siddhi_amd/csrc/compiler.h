// Host compiler: SiddhiQL AST → device plan (plan.h). Lowering mirrors
// core/util/parser/StateInputStreamParser.java:78-432 (state tables, within lists, every/next edges,
// receivers), SelectorParser.java:140-200 (projections) and ExpressionParser.java:231-1371 (bytecode).
#pragma once
#include <string>
#include <unordered_map>
#include <vector>

#include "plan.h"
#include "siddhiql/ast.h"

namespace sm {

struct Dict {  // string dictionary: device columns carry int32 ids
  std::unordered_map<std::string, int32_t> ids;
  std::vector<std::string> strs;
  int32_t intern(const std::string& s) {
    auto it = ids.find(s);
    if (it != ids.end()) return it->second;
    int32_t id = (int32_t)strs.size();
    strs.push_back(s);
    ids.emplace(s, id);
    return id;
  }
};

struct CompiledQuery {
  std::string name;
  std::string insert_into;
  int order = 0;          // position in app.order
  int partition = -1;     // partition index, -1 = none
  DQuery hdr{};
  std::vector<char> blob;               // header + tables, uploaded once
  std::vector<int32_t> sel_types;       // output attribute types
  std::vector<std::string> sel_names;
  std::vector<int> streams;             // app stream indices the query consumes
  bool has_absent = false;
  // fast path: every e1=S[c1] -> e2=S[c2] within T (closed form)
  bool fast_every_within = false;
  int64_t fast_within = -1;             // -1 = no within
  int fast_c1_off = 0, fast_c1_len = 0; // program over e1's stream columns (stream context)
  int fast_c2_off = 0, fast_c2_len = 0; // program over (e1 slot 0, e2 slot 1) state context
};

struct CompiledPartition {
  std::vector<int> streams;                    // partitioned stream indices
  std::vector<std::vector<Instr>> key_code;    // per partitioned stream: key expression program
  std::vector<std::vector<DVal>> key_consts;
  std::vector<int32_t> key_type;               // result type per stream
};

// Compile one query. `app_streams` gives stream index by id. Throws sql::*Error.
CompiledQuery compile_query(const sql::App& app, const sql::Query& q, int order, int partition, Dict& dict);
CompiledPartition compile_partition(const sql::App& app, const sql::Partition& p, Dict& dict);

int stream_index(const sql::App& app, const std::string& id);

}  // namespace sm
