// SiddhiQL subset AST (hot-path scope: define stream, partition, filter / pattern / sequence queries,
// select, insert into, @app:playback, @info(name)).
//
// Mirrors the shapes of siddhi-query-api:
//   StateInputStream            modules/siddhi-query-api/.../execution/query/input/stream/StateInputStream.java:16
//   Stream/Absent/Next/Every/Logical/CountStateElement
//                               modules/siddhi-query-api/.../execution/query/input/state/*.java
//   Expression tree             modules/siddhi-query-api/.../expression/**
// Shared by the product compiler (siddhi_amd/csrc/compiler.cpp) and the CPU oracle (oracle/cpu_ref.cpp);
// each lowers the AST independently.
#pragma once
#include <cstdint>
#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

namespace sql {

enum class AttrType : int { INT = 0, LONG = 1, FLOAT = 2, DOUBLE = 3, STRING = 4, BOOL = 5 };

inline const char* attr_type_name(AttrType t) {
  switch (t) {
    case AttrType::INT: return "INT";
    case AttrType::LONG: return "LONG";
    case AttrType::FLOAT: return "FLOAT";
    case AttrType::DOUBLE: return "DOUBLE";
    case AttrType::STRING: return "STRING";
    case AttrType::BOOL: return "BOOL";
  }
  return "?";
}

// Index constants, SiddhiConstants.java:79-83 (CURRENT = -1, LAST = -2, ANY = -1).
constexpr int kCurrent = -1;
constexpr int kLast = -2;
constexpr int kAny = -1;
constexpr int kNoIndex = INT32_MIN;  // variable without [index]

struct ParseError : std::runtime_error {
  using std::runtime_error::runtime_error;
};
struct ValidationError : std::runtime_error {
  using std::runtime_error::runtime_error;
};
struct UnsupportedError : std::runtime_error {
  using std::runtime_error::runtime_error;
};

struct Attribute {
  std::string name;
  AttrType type;
};

struct StreamDef {
  std::string id;  // "#name" for a partition's inner stream
  std::vector<Attribute> attrs;
  // defined by a query's `insert into` (SiddhiApp.defineStream from the query's output attributes) rather than by
  // `define stream`; partition = the partition an inner stream belongs to (-1: app-level stream)
  bool implicit = false;
  int partition = -1;
  int index_of(const std::string& n) const {
    for (size_t i = 0; i < attrs.size(); ++i)
      if (attrs[i].name == n) return (int)i;
    return -1;
  }
};

// INSTANCE_OF: instanceOf<Type>(x) (core/executor/function/InstanceOf*FunctionExecutor.java); ctype = the tested type
enum class ExprKind { CONST, VAR, AND, OR, NOT, CMP, MATH, IS_NULL, INSTANCE_OF };
enum class CmpOp { EQ, NE, LT, LE, GT, GE };
enum class MathOp { ADD, SUB, MUL, DIV, MOD };

struct Expr {
  ExprKind kind;
  // CONST
  AttrType ctype = AttrType::INT;
  bool cnull = false;
  int64_t ival = 0;
  double dval = 0.0;
  std::string sval;
  // VAR: [streamRef[index].]attr
  std::string stream_ref;   // event reference (e1) or stream id; empty = bare attribute
  int index = kNoIndex;     // attribute_index as the visitor returns it (LAST - k for last-k)
  std::string attr;
  // CMP / MATH
  CmpOp cmp = CmpOp::EQ;
  MathOp math = MathOp::ADD;
  std::vector<std::unique_ptr<Expr>> ch;
};
using ExprP = std::unique_ptr<Expr>;

enum class StateKind { STREAM, ABSENT, NEXT, EVERY, LOGICAL, COUNT };
enum class LogicalType { AND, OR };

struct StateElem {
  StateKind kind;
  bool has_within = false;
  int64_t within_ms = 0;
  // STREAM / ABSENT
  std::string event_ref;       // e1 (may be empty)
  std::string stream_id;
  std::vector<ExprP> filters;  // S[f1][f2] ...
  bool has_wait = false;       // ABSENT: 'for <time>' present
  int64_t wait_ms = 0;
  // NEXT: a -> b ; EVERY: a ; LOGICAL: a (element1) op b (element2) ; COUNT: a
  std::unique_ptr<StateElem> a, b;
  LogicalType ltype = LogicalType::AND;
  int min_count = kAny, max_count = kAny;
};
using StateP = std::unique_ptr<StateElem>;

enum class InputKind { SINGLE, PATTERN, SEQUENCE };

struct OutputAttr {
  ExprP expr;
  std::string rename;
};

struct Query {
  std::string name;  // @info(name=...) or generated "query_<n>"
  InputKind input = InputKind::SINGLE;
  // SINGLE
  std::string stream_id;
  std::vector<ExprP> filters;
  // PATTERN / SEQUENCE
  StateP state;
  // selection
  bool select_all = false;
  std::vector<OutputAttr> select;
  ExprP having;  // query_section 'having' (SiddhiQL.g4 having: HAVING expression); null = none
  std::string insert_into;  // output stream
  int output_event_type = 0;  // 0 = current events (only supported type)
};

struct PartitionWith {
  std::string stream_id;
  ExprP key;  // attribute expression, evaluated on the stream's event
};

struct Partition {
  std::vector<PartitionWith> with;
  std::vector<Query> queries;
};

struct App {
  std::string name;
  bool playback = false;
  std::vector<StreamDef> streams;
  std::vector<Query> queries;        // non-partitioned
  std::vector<Partition> partitions;
  // Query order across the whole app (for output interleaving): (partition idx or -1, query idx)
  std::vector<std::pair<int, int>> order;
  const StreamDef* find_stream(const std::string& id) const {
    for (auto& s : streams)
      if (s.id == id) return &s;
    return nullptr;
  }
};

// Parses SiddhiQL text; throws ParseError / ValidationError / UnsupportedError.
App parse_app(const std::string& text);

// Canonical JSON of a parsed app (siddhiql/dump.cpp; shapes documented there).
std::string dump_app_json(const App& a);

// Utility: all stream ids referenced in a state tree in StateInputStream.collectStreamIds order
// (StateInputStream.java:70-88; absent elements are StreamStateElements and are included).
void collect_stream_ids(const StateElem* e, std::vector<std::string>& out);

}  // namespace sql
