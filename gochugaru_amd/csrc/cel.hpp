// cel.hpp — host-side caveat evaluation: a CEL subset with partial evaluation, and the JSON
// values caveat contexts are written in.
//
// SpiceDB evaluates a caveated relationship's CEL expression over the relationship's stored
// context merged with the check-time context (CheckBulkPermissionsRequestItem.Context, sent by
// Client.Check at client/client.go:257 from rel.Relationship.MustV1ProtoCaveat,
// rel/relationship.go:174-188). A parameter missing from both leaves the expression unknown
// and the check CONDITIONAL. The graph walk stays on the GPU: the host
// evaluates each distinct (caveat instance, check context) pair once per batch and hands the
// device a table of their outcomes (engine.hip cav_state).
#pragma once
#include <cstdint>
#include <map>
#include <memory>
#include <string>
#include <vector>

namespace gck {
namespace cel {

struct Value {
  // TS (timestamp) and DUR (duration) hold microseconds in `i`; IP holds the 4 or 16 address
  // bytes in `s`
  enum Kind : uint8_t { UNKNOWN, NUL, BOOL, INT, DBL, STR, LIST, MAP, TS, DUR, IP } k = UNKNOWN;
  bool b = false;
  int64_t i = 0;
  double d = 0;
  std::string s;
  std::shared_ptr<const std::vector<Value>> l;
  std::shared_ptr<const std::map<std::string, Value>> m;
};

using Object = std::map<std::string, Value>;

// Parses a JSON object (a caveat context); "" parses as the empty object. Throws
// Error(GCK_E_INVALID_ARGUMENT) on malformed input or a non-object top-level value.
Object parse_context(const std::string& json);

struct Node;

// Compiles a caveat body (the CEL text between the braces of `caveat name(...) { ... }`).
// `params` (name, declared type): a parameter declared timestamp / duration / ipaddress takes
// its context value as text (RFC 3339, Go duration syntax, an IPv4/IPv6 address) and is
// converted on lookup. Throws Error(GCK_E_SCHEMA).
std::shared_ptr<const Node> compile(const std::string& body,
                                    const std::vector<std::pair<std::string, std::string>>& params = {});

enum Outcome : uint8_t { FALSE = 0, TRUE = 1, PARTIAL = 2 };

// Evaluates `expr` with the relationship's stored context taking precedence over the check
// context (either may be null). TRUE only for the boolean true; PARTIAL when the value depends
// on a missing parameter. Throws Error(GCK_E_INVALID_ARGUMENT) on an evaluation error.
Outcome evaluate(const Node& expr, const Object* stored, const Object* check);

}  // namespace cel
}  // namespace gck
