"""Hand-derived LookupSubjects answers with wildcard grants (SpiceDB reports `user:*` as the
subject "*"; client/client.go:560-599 yields its SubjectObjectId). Shared by the oracle test
(tests/test_oracle.py) and the GPU test (tests/test_gpu_lookup.py)."""

WILD_SCHEMA = """
definition user {}
definition group { relation member: user | user:* }
caveat tuesday(day string) { day == "tuesday" }
definition doc {
  relation viewer: user | user:* | user:* with tuesday | group#member
  relation banned: user
  relation member: user
  permission view = viewer
  permission view_unbanned = viewer - banned
  permission view_member = viewer & member
}
"""

WILD_CASES = [
    # (tuples, permission, subject kind, expected (subject, permissionship) pairs)
    (["doc:d#viewer@user:*", "doc:d#viewer@user:tom"], "view", "user", [("*", 2), ("tom", 2)]),
    (["doc:d#viewer@user:*"], "view", "user", [("*", 2)]),
    (["doc:d#viewer@user:*", "doc:d#banned@user:bob", "doc:d#viewer@user:bob"], "view_unbanned", "user", [("*", 2)]),
    (["doc:d#viewer@user:*", "doc:d#member@user:tom", "doc:d#member@user:ann"], "view_member", "user",
     [("ann", 2), ("tom", 2)]),
    (["doc:d#viewer@user:*[tuesday]", "doc:d#viewer@user:tom"], "view", "user", [("*", 3), ("tom", 2)]),
    (["doc:d#viewer@group:g#member", "group:g#member@user:*", "group:g#member@user:amy"], "view", "user",
     [("*", 2), ("amy", 2)]),
    (["doc:d#viewer@group:g#member", "group:g#member@user:*"], "view", "group#member", [("g", 2)]),
    (["doc:d#viewer@user:ann", "doc:d#banned@user:ann"], "view_unbanned", "user", []),
]
