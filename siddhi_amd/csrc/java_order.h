// Java 8 orders the partition runtime depends on (host side).
//
// PartitionStreamReceiver.send(ComplexEvent) (core/partition/PartitionStreamReceiver.java:271-275) hands an event
// of a stream the partition does not key to every partition instance by iterating
// cachedStreamJunctionMap.values(), a ConcurrentHashMap<String, StreamJunction> keyed by streamId + key
// (:53, addStreamJunction :284-300, filled in instance creation order by PartitionRuntime.clonePartition
// :262-309 → updatePartitionStreamReceivers :311-315). That iteration order is deterministic: it is a function of
// the keys' String.hashCode and the order they were put. JavaChmOrder restates the single-threaded put and
// values() traversal of java.util.concurrent.ConcurrentHashMap (Java 8): spread hash, table of 16 created on the
// first put, resize at 0.75 load (transfer: each bin split into the i / i + n bins by the lastRun rule, nodes
// before the run prepended), bins of 8+ nodes turned into TreeBins once the table has 64 bins (tryPresize first,
// below that), TreeBin puts prepended to its `first` list, TreeBins of 6 or fewer nodes untreeified at a split.
#pragma once
#include <cstdint>
#include <string>
#include <vector>

namespace sm {

// String.hashCode of a UTF-8 string (over its UTF-16 code units)
int32_t java_string_hash(const std::string& utf8);
// String.valueOf of a partition key value (ValuePartitionExecutor.execute :34-40): the key part of the junction
// id. type = T_INT / T_LONG / T_FLOAT / T_DOUBLE / T_BOOL; strings are passed as themselves.
std::string java_value_string(int type, int64_t code);

class JavaChmOrder {
 public:
  // put of a key that is not in the map yet
  void put(const std::string& key);
  // insertion indices of the keys in values() iteration order
  std::vector<int> order() const;
  size_t size() const { return hash_.size(); }

 private:
  struct Bin {
    bool tree = false;
    std::vector<int> nodes;  // insertion indices in list order (a TreeBin: its `first` list)
  };
  std::vector<Bin> tab_;
  std::vector<int32_t> hash_;  // spread hash of each key, by insertion index
  int64_t size_ctl_ = 0;
  void transfer();
  void try_presize(int64_t size);
};

}  // namespace sm
