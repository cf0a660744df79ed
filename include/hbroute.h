/*
 * hbroute.h — host owner routing of raft messages across the GPUs of a node
 * (SURVEY.md §8(e)), part of libhbnode.so.
 *
 * Groups never interact (raft/multinode.go:125-131), so a node with N GPUs
 * runs N independent engines, one per GPU: group id g belongs to rank
 * splitmix64(g) % N and lives at a dense local slot there.  Every message a
 * node receives for a group (what multiNode.Step hands to its run goroutine,
 * raft/multinode.go:233-237, 369-381) must reach the engine that owns the
 * group, in arrival order.  The router does that for a whole arrival-ordered
 * stream in one pass, on host threads: per rank, the positions of its
 * messages in the stream and their local slots (the hb_batch.group values of
 * that rank's engine), order kept.  No torch / C++ types: plain pointers.
 *
 * Python mirror and oracle: etcd_amd/shard.py (ShardMap.route_local), which
 * tests/test_route.py checks this library against.
 */
#ifndef HBROUTE_H_
#define HBROUTE_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct hbn_router hbn_router;

/* The owner of a group id: splitmix64(id) % world (world 1: rank 0). */
uint32_t hbn_owner(uint64_t group_id, uint32_t world);

/* A router over the node's groups: ids[0 .. n) (distinct), each owned by rank
 * hbn_owner(id, world) at local slot = its position among that rank's ids in
 * the order given (etcd_amd/shard.py ShardMap.local_ids).  A dense id space
 * (every id < 2 n + 1024) is looked up in a flat table, any other through an
 * open-addressing hash.  threads: host threads for hbn_route (0 = min(16,
 * cores)).  Returns HB_EINVAL (-1) on a duplicate id, world 0 or above 255,
 * or a rank owning more than 2^24 groups (an engine's capacity, hb_create);
 * HB_ENOMEM (-2) when the tables cannot be allocated.  No router function
 * lets a C++ exception out: hbn_route / hbn_route_take return HB_ENOMEM when
 * host memory runs out. */
int hbn_router_create(const uint64_t* ids, uint64_t n, uint32_t world, uint32_t threads, hbn_router** out);
int hbn_router_destroy(hbn_router* r);
/* Groups owned by `rank` (its engine's capacity), and their global ids by slot. */
uint64_t hbn_router_local_count(const hbn_router* r, uint32_t rank);
int hbn_router_local_ids(const hbn_router* r, uint32_t rank, uint64_t* ids /* [local_count] */);

/* Route an arrival-ordered stream of group ids: one pass over the stream
 * looks every id up (the router keeps each message's rank and slot, 4 bytes,
 * until the next hbn_route) and sets counts[k] = the messages of rank k;
 * *unknown (may be NULL) = the messages for group ids the router does not
 * know, which go nowhere (multiNode.Step of a missing group).  Then
 * hbn_route_take writes, for each rank k whose pos[k] / slot[k] is non-NULL
 * (arrays of at least counts[k]; pos or slot may be NULL as a whole),
 * pos[k][j] = the stream position of rank k's j-th message and slot[k][j] its
 * local slot (the hb_batch.group value of that rank's engine), in arrival
 * order.  A router is used by one thread at a time. */
int hbn_route(hbn_router* r, const uint64_t* gids, uint64_t n, uint64_t* counts /* [world] */, uint64_t* unknown);
int hbn_route_take(hbn_router* r, uint64_t* const* pos /* [world] or NULL */, uint32_t* const* slot /* [world] or NULL */);

#ifdef __cplusplus
}
#endif
#endif /* HBROUTE_H_ */
