// minisched.h — C++ host mirror of minisched's scheduling loop above the C ABI.
//
// The reference (Go, /root/reference/minisched) cannot be built here, so the
// host side of the drop-in is restated in C++ with the reference's names,
// argument meaning and error behaviour:
//   v1 objects / tolerations          k8s.io/api v0.22.0 (restated)
//   framework types, ClusterEvent     k8s@v1.22.0 pkg/scheduler/framework (restated)
//   SchedulingQueue                   minisched/queue/queue.go
//   plugin registry + events          minisched/initialize.go:80-213
//   Scheduler::ScheduleOne/ErrorFunc  minisched/minisched.go:32-113, :283-298
//   node/pod event handlers           minisched/eventhandler.go:14-90
// The filter/score/selectHost work runs on the GPU through ms_schedule_batch
// (include/minisched_gpu.h); there is no CPU implementation of it here.
#pragma once

#include <chrono>
#include <tuple>
#include <cstdint>
#include <deque>
#include <functional>
#include <map>
#include <memory>
#include <optional>
#include <set>
#include <string>
#include <vector>

#include "minisched_gpu.h"

namespace minisched {

// ---------------------------------------------------------------- v1 (subset)
namespace v1 {

constexpr const char *kTaintNodeUnschedulable = "node.kubernetes.io/unschedulable";
constexpr const char *kTaintEffectNoSchedule = "NoSchedule";

struct Taint {
    std::string key, value, effect;
};

struct Toleration {
    std::string key;
    std::string op;  // "" (== Equal), "Equal", "Exists"
    std::string value;
    std::string effect;
    // core/v1 Toleration.ToleratesTaint (k8s.io/api v0.22.0)
    bool ToleratesTaint(const Taint &t) const;
};

bool TolerationsTolerateTaint(const std::vector<Toleration> &tols, const Taint &t);

// Quantities already normalised: cpu in millicores, memory in bytes. `other`
// holds every other resource name (ephemeral-storage, hugepages-*, extended
// resources such as amd.com/gpu): upstream Fit.fitsRequest checks the ones a
// pod requests, ms_pod_rec cannot carry them, so a pod requesting any is
// refused under NodeResourcesFit (UnsupportedRequest); on nodes they are ignored
// (no admitted pod requests them, so Requested stays 0 and no decision reads them).
struct ResourceList {
    std::optional<int64_t> cpu_milli, memory, pods;
    std::map<std::string, int64_t> other;
};

struct Container {
    std::string name;
    ResourceList requests;
};

struct Pod {
    std::string name, ns = "default", uid;
    std::string node_name;  // Spec.NodeName (assigned pods are not queued)
    std::vector<Toleration> tolerations;
    std::vector<Container> containers, init_containers;
    std::optional<ResourceList> overhead;
};

struct Node {
    std::string name;
    bool unschedulable = false;  // Spec.Unschedulable
    ResourceList allocatable;    // Status.Allocatable
};

}  // namespace v1

// ------------------------------------------------------------ framework subset
namespace framework {

enum class Code { Success = 0, Error = 1, Unschedulable = 2, UnschedulableAndUnresolvable = 3, Wait = 4, Skip = 5 };

// ActionType bits, k8s@v1.22.0 framework/types.go
enum ActionType : uint32_t {
    Add = 1u << 0,
    Delete = 1u << 1,
    UpdateNodeAllocatable = 1u << 2,
    UpdateNodeLabel = 1u << 3,
    UpdateNodeTaint = 1u << 4,
    UpdateNodeCondition = 1u << 5,
    All = (1u << 6) - 1,
    Update = UpdateNodeAllocatable | UpdateNodeLabel | UpdateNodeTaint | UpdateNodeCondition,
};

using GVK = std::string;  // "Pod", "Node", ... ; "*" is the wildcard
constexpr const char *kPod = "Pod";
constexpr const char *kNode = "Node";
constexpr const char *kWildCard = "*";

struct ClusterEvent {
    GVK resource;
    uint32_t action = 0;
    std::string label;
    bool IsWildCard() const { return resource == kWildCard && action == All; }
    bool operator<(const ClusterEvent &o) const {
        return std::tie(resource, action, label) < std::tie(o.resource, o.action, o.label);
    }
};

struct Diagnosis {
    std::set<std::string> UnschedulablePlugins;
};

// Result of one scheduling cycle as the reference's error handling sees it.
struct ScheduleError {
    bool fit_error = false;  // *framework.FitError vs plain error
    Diagnosis diagnosis;
    std::string message;
};

struct QueuedPodInfo {
    v1::Pod pod;
    std::chrono::steady_clock::time_point timestamp{}, initial_attempt_timestamp{};
    int attempts = 0;
    std::set<std::string> UnschedulablePlugins;
};

}  // namespace framework

// --------------------------------------------------------------------- plugins
// GPU twins: Name() and EventsToRegister() drive queue/event registration
// exactly as in the reference; their Filter/Score bodies run on the device.
struct Plugin {
    virtual ~Plugin() = default;
    virtual std::string Name() const = 0;
    virtual std::vector<framework::ClusterEvent> EventsToRegister() const = 0;
};

struct NodeUnschedulable : Plugin {  // k8s@v1.22.0 nodeunschedulable
    std::string Name() const override { return "NodeUnschedulable"; }
    std::vector<framework::ClusterEvent> EventsToRegister() const override;
};
struct NodeNumber : Plugin {  // minisched/plugins/score/nodenumber/nodenumber.go
    std::string Name() const override { return "NodeNumber"; }
    std::vector<framework::ClusterEvent> EventsToRegister() const override;  // nodenumber.go:66-70
};
struct NodeResourcesFit : Plugin {  // k8s@v1.22.0 noderesources.Fit (LeastAllocated scoring)
    std::string Name() const override { return "NodeResourcesFit"; }
    std::vector<framework::ClusterEvent> EventsToRegister() const override;
};

// ----------------------------------------------------------------------- queue
// minisched/queue/queue.go, including its quirks: NextPod is FIFO over
// activeQ; AddUnschedulable refreshes Timestamp; Attempts is never
// incremented (so backoff is always 1 s); backoffQ is never flushed.
class SchedulingQueue {
   public:
    using Clock = std::function<std::chrono::steady_clock::time_point()>;
    explicit SchedulingQueue(std::map<framework::ClusterEvent, std::set<std::string>> cluster_event_map,
                             Clock clock = nullptr);

    void Add(const v1::Pod &pod);                                        // queue.go:35-43
    std::optional<v1::Pod> NextPod();                                    // queue.go:84-92 (non-blocking)
    void AddUnschedulable(framework::QueuedPodInfo pinfo);               // queue.go:95-107
    void MoveAllToActiveOrBackoffQueue(const framework::ClusterEvent &e);  // queue.go:54-82

    size_t ActiveLen() const { return active_.size(); }
    size_t BackoffLen() const { return backoff_.size(); }
    size_t UnschedulableLen() const { return unschedulable_.size(); }
    const framework::QueuedPodInfo *Unschedulable(const std::string &key) const;
    static std::string KeyFunc(const v1::Pod &p) { return p.name + "_" + p.ns; }  // queue.go:152-154

    bool PodMatchesEvent(const framework::QueuedPodInfo &pinfo, const framework::ClusterEvent &e) const;
    bool IsPodBackingoff(const framework::QueuedPodInfo &pinfo) const;
    static std::chrono::nanoseconds CalculateBackoffDuration(const framework::QueuedPodInfo &pinfo);

   private:
    std::deque<framework::QueuedPodInfo> active_;
    std::vector<framework::QueuedPodInfo> backoff_;
    std::map<std::string, framework::QueuedPodInfo> unschedulable_;
    std::map<framework::ClusterEvent, std::set<std::string>> event_map_;
    Clock clock_;
    std::chrono::steady_clock::time_point Now() const;
};

// ------------------------------------------------------------------- scheduler
struct ScheduleResult {
    enum Kind { NoPod, Scheduled, Unschedulable, Error } kind = NoPod;
    std::string pod, node;
    int64_t score = 0;
    framework::ScheduleError error;
};

// Record encoders (what the cgo shim computes per object).
int NameDigit(const std::string &name);  // strconv.Atoi(name[len-1:]) : 0..9 or -1
ms_pod_rec EncodePod(const v1::Pod &pod, uint32_t ordinal);
// The first request name of a container, init container or the overhead that
// ms_pod_rec cannot carry ("" if none). Under NodeResourcesFit such a pod gets
// a plain Error from ScheduleOne and never reaches the device.
std::string UnsupportedRequest(const v1::Pod &pod);

// Node ordinals aligned to the name digit: a node whose name ends in digit d
// gets an ordinal with ordinal % 10 == d (the lowest free one), so every 30
// consecutive ordinals hold at most 3 nodes of one digit whatever the informer
// Add order — the layout K1 pp's three fast hash slots cover.
// The ordinal is an internal handle: the tie-break is a pure function of
// (seed, pod, ordinal), uniform over tied nodes whichever ordinals they hold.
// Names without a digit never score NodeNumber's 10 and fill the lowest free
// ordinal of any residue. When a digit's residue is full up to the capacity,
// its nodes take the lowest free ordinal of any residue (correct, on the
// kernel's bit-scan path).
// Digit-aligned ordinals, within a bounded spread: a digit-aligned slot is taken
// only while it stays below kSpreadSlack + 2 x (live nodes + 1); past that (e.g.
// every node name ending in '0', which digit alignment would spread over 10x
// the ordinals) the lowest free ordinal of any residue is used, so the sweep
// extent (HighWater) stays within about twice the live node count.
class OrdinalAllocator {
   public:
    static constexpr uint32_t kSpreadSlack = 300;  // 10 groups of 30 ordinals
    // Skew fallback (encode.DigitOrdinals in lockstep): with at
    // least kSkewMinLive live nodes and 10 x the largest digit share above 2.6
    // (100 x max count > kSkewBreakEvenX10 x live), an aligned table costs more
    // to sweep than a dense one on the bit-scan path, so allocations go dense.
    static constexpr uint32_t kSkewMinLive = 100;
    static constexpr uint32_t kSkewBreakEvenX10 = 26;
    explicit OrdinalAllocator(uint32_t capacity);
    uint32_t Allocate(int digit);  // digit 0..9, or -1; throws std::length_error when full
    void Release(uint32_t ordinal, int digit);  // digit: the released node's name digit
    uint32_t HighWater() const;    // 1 + the highest ordinal ever handed out (0 if none)
    bool Skewed() const;           // allocations currently go dense

   private:
    uint32_t LowestAny();
    uint32_t Pick(int digit);
    uint32_t cap_;
    uint32_t live_ = 0;
    uint32_t count_[10] = {};      // live nodes per name digit
    uint32_t next_[10];            // lowest never-used ordinal of residue d
    std::set<uint32_t> free_[10];  // released ordinals per residue
    uint32_t high_ = 0;
};
struct NodeUsage {  // NodeInfo.Requested / NonZeroRequested / len(Pods)
    int64_t req_cpu = 0, req_mem = 0, nz_cpu = 0, nz_mem = 0;
    int32_t pods = 0;
};
ms_node_rec EncodeNode(const v1::Node &node, const NodeUsage &usage);

class Scheduler {
   public:
    enum class PluginSet { NU_NN = MS_PLUGINS_NU_NN, NU_NRF_NN_LA = MS_PLUGINS_NU_NRF_NN_LA };
    // Binds a pod (minisched.go:266-277); returning false re-queues it.
    using Binder = std::function<bool(const v1::Pod &, const std::string &node)>;

    struct Options {
        PluginSet plugins = PluginSet::NU_NN;
        int device = 0;
        uint32_t max_nodes = 1u << 16;
        uint64_t seed = 1;
        SchedulingQueue::Clock clock = nullptr;
        Binder binder = nullptr;
    };

    // minisched.New (initialize.go:35-78): builds plugin slices, event map,
    // queue; creates the device context. Throws std::runtime_error with
    // ms_last_error() text when the device context cannot be created.
    explicit Scheduler(const Options &opt);
    ~Scheduler();
    Scheduler(const Scheduler &) = delete;
    Scheduler &operator=(const Scheduler &) = delete;

    // eventhandler.go: unassigned pods are queued; node Add/Update/Delete push
    // device deltas, then move unschedulable pods (registered actions only).
    void OnPodAdd(const v1::Pod &pod);
    void OnNodeAdd(const v1::Node &node);
    void OnNodeUpdate(const v1::Node &old_node, const v1::Node &new_node);
    void OnNodeDelete(const v1::Node &node);

    // One scheduling cycle (minisched.go:32-113) for the next queued pod.
    ScheduleResult ScheduleOne();
    // Up to k queued pods in queue order in one device call (sequential mode,
    // identical placements to k ScheduleOne calls).
    std::vector<ScheduleResult> ScheduleBatch(size_t k);

    SchedulingQueue &Queue() { return *queue_; }
    const std::vector<std::unique_ptr<Plugin>> &FilterPlugins() const { return filter_; }
    const std::vector<std::unique_ptr<Plugin>> &ScorePlugins() const { return score_; }
    const std::map<framework::ClusterEvent, std::set<std::string>> &EventMap() const { return event_map_; }
    uint32_t Gvk(const std::string &gvk) const;  // unionedGVKs (initialize.go:169-179)
    const NodeUsage *Usage(const std::string &node) const;
    ms_ctx *Ctx() const { return ctx_; }

   private:
    void ErrorFunc(const v1::Pod &pod, const framework::ScheduleError &err);  // minisched.go:283-298
    uint32_t NodeOrdinal(const std::string &name, bool create);
    ScheduleResult Finish(const v1::Pod &pod, const ms_pod_rec &rec, const ms_result &r);

    Options opt_;
    ms_ctx *ctx_ = nullptr;
    std::vector<std::unique_ptr<Plugin>> filter_, score_;
    std::map<framework::ClusterEvent, std::set<std::string>> event_map_;
    std::map<std::string, uint32_t> gvk_map_;
    std::unique_ptr<SchedulingQueue> queue_;
    std::map<std::string, uint32_t> ordinal_;  // node name -> global ordinal
    std::vector<std::string> names_;           // ordinal -> node name ("" when free)
    OrdinalAllocator ordinals_;                // digit-aligned node ordinals
    std::map<std::string, v1::Node> nodes_;
    std::map<std::string, NodeUsage> usage_;
    std::map<std::string, uint32_t> pod_ordinal_;
    uint32_t next_pod_ordinal_ = 0;
};

}  // namespace minisched
