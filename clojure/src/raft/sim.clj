(ns raft.sim
  "Batched MI355X simulation of raft.core's node loop (src/raft/core.clj:176-203 of the reference)
  through libraftsim.so, the C ABI of include/raftsim.h (ABI version 2). One handle simulates
  n-clusters independent clusters of `nodes` nodes each on `n-devices` GPUs; a node is the map
  init-node builds (core.clj:31-38) and every `wait` iteration of every node happens inside step!.
  Semantics: SIM_SPEC.md. JNA, because Clojure 1.6 predates Panama (JDK 22)."
  (:import [com.sun.jna NativeLibrary Memory Pointer Function]
           [com.sun.jna.ptr PointerByReference]))

(def ^:private lib (delay (NativeLibrary/getInstance "raftsim")))

(defn- f ^Function [fname] (.getFunction ^NativeLibrary @lib fname))

(defn- last-error [] (.getString ^Pointer (.invokePointer (f "raft_sim_last_error") (object-array [])) 0))

(defn- check
  "raft_sim_* calls return 0 or a negative errno (include/raftsim.h); never throw across the ABI."
  [rc]
  (when (neg? rc) (throw (ex-info (last-error) {:rc rc})))
  rc)

(defn- call [fname & args] (check (.invokeInt (f fname) (object-array args))))

(def abi-version 2)

;; raft_sim_config_t (120 bytes): u32 fields, the u64 seed at 24, i32 device and n_devices
(def config-offsets
  {:n-clusters 0 :cluster-offset 4 :nodes 8 :log-cap 12 :arena-cap 16 :inbox-cap 20 :seed 24
   :hb 32 :el-base 36 :el-span 40 :drop-ppm 44 :dup-ppm 48 :dmin 52 :dmax 56 :part-ppm 60
   :part-epoch 64 :client-ppm 68 :variant-flags 72 :device 76 :ticks-per-launch 80
   :commit-stream-cap 84 :trace-cap 88 :trace-entry-cap 92 :schedule 96 :client-period 100
   :client-burst 104 :client-redirects 108 :n-devices 112})
(def config-size 120)

;; raft_node_t (136 bytes)
(def node-offsets
  {:role 0 :voted-for 1 :leader-id 2 :fault 3 :entries-is-seq 4 :ls-present 5 :votes 6 :ls-keys 8
   :current-term 12 :commit-index 16 :log-len 20 :deadline 24 :next-index 28 :match-index 64
   :last-led-term 100 :arena-base 104 :arena-frontier 108 :req-count 112 :res-count 116
   :commit-count 120 :trace-hash 128})
(def node-size 136)

;; raft_counters_t (248 bytes): node_ticks, first_violation_tick, 28 sums, payload_max
(def counter-names
  [:ev-rv :ev-ae :ev-cs :ev-vr :ev-ar :ev-timeout :ev-heartbeat :leaders :sent :delivered :dropped
   :partitioned :duplicated :overflow :to-halted :client-injected :halt-ioobe :halt-npe :halt-cce
   :halt-overflow :entries-appended :entries-applied :payload-evicted :viol-election :viol-log
   :viol-complete :redirects :client-abandoned])
(def counters-size 248)

(def ^:private states [:follower :candidate :leader :follwer])   ; :follwer is core.clj:76's typo
(def ^:private halts {1 :index-out-of-bounds 2 :null-pointer 3 :class-cast 4 :log-capacity})

(defn create
  "Like (component/start (raft-system id cluster)) (core.clj:23-29,201) for every node of
  n-clusters clusters. cfg keys: config-offsets; absent keys keep raft_sim_default_config."
  [cfg]
  (let [m (Memory. config-size)]
    (.invokeVoid (f "raft_sim_default_config") (object-array [m]))
    (doseq [[k v] cfg :let [off (config-offsets k)]]
      (when-not off (throw (ex-info "unknown config key" {:key k})))
      (if (= k :seed) (.setLong m off (long v)) (.setInt m off (unchecked-int v))))
    (let [out (PointerByReference.)]
      (call "raft_sim_create" m out)
      {:ptr (.getValue out) :nodes (int (:nodes cfg 5))})))

(defn step!
  "(loop [node ...] (recur (wait system node))) of core.clj:202-203, `ticks` times, for all nodes."
  [sim ticks]
  (call "raft_sim_step" (:ptr sim) (int ticks))
  sim)

(defn tick [sim] (.invokeLong (f "raft_sim_tick") (object-array [(:ptr sim)])))

(defn set-tick!
  "Resume at `t` after restoring state through the write calls (deadlines are absolute ticks)."
  [sim t]
  (call "raft_sim_set_tick" (:ptr sim) (long t))
  sim)

(defn nodes
  "The node maps of cluster c, shaped like init-node (core.clj:31-38), plus :halted."
  [sim c]
  (let [n (:nodes sim)
        m (Memory. (* node-size n))
        ids (fn [mask] (set (filter #(bit-test mask %) (range 1 (inc n)))))]
    (call "raft_sim_read_nodes" (:ptr sim) (int c) (int 1) m)
    (vec (for [i (range n)
               :let [b (* i node-size)
                     at (fn [k] (+ b (node-offsets k)))
                     ls-keys (ids (.getShort m (at :ls-keys)))
                     peer-map (fn [k] (into {} (for [p ls-keys]
                                                 [p (.getInt m (+ (at k) (* 4 (dec p))))])))]]
           {:id (inc i)
            :state (states (.getByte m (at :role)))
            :current-term (.getInt m (at :current-term))
            :voted-for (let [v (.getByte m (at :voted-for))] (when (pos? v) v))
            :leader-id (let [v (.getByte m (at :leader-id))] (when (pos? v) v))
            :leader-state (when (pos? (.getByte m (at :ls-present)))
                            {:next-index (peer-map :next-index)
                             :match-index (peer-map :match-index)})
            :votes (ids (.getShort m (at :votes)))
            :halted (halts (.getByte m (at :fault)))}))))

(defn log-entries
  "The Log atom's :entries of node `id` of cluster c (log.clj:33-34), as {:term t :val v} maps."
  [sim c id]
  (let [node (Memory. (* node-size (:nodes sim)))
        _ (call "raft_sim_read_nodes" (:ptr sim) (int c) (int 1) node)
        b (* (dec id) node-size)
        base (.getInt node (+ b (node-offsets :arena-base)))
        len (.getInt node (+ b (node-offsets :log-len)))
        cap (call "raft_sim_read_arena" (:ptr sim) (int c) (int id) nil (int 0))
        ar (Memory. (* 8 cap))]
    (call "raft_sim_read_arena" (:ptr sim) (int c) (int id) ar (int cap))
    (vec (for [i (range len) :let [s (* 8 (mod (+ base i) cap))]]
           {:term (.getInt ar s) :val (.getInt ar (+ s 4))}))))

(defn commit-log
  "What apply-entries! wrote to node_<id>.log (log.clj:16-18,69-76), newest commit_stream_cap."
  [sim c id cap]
  (let [m (Memory. (* 4 (max 1 cap)))
        n (call "raft_sim_read_commit_stream" (:ptr sim) (int c) (int id) m (int cap))]
    (vec (for [i (range n)] (.getInt m (* 4 i))))))

(defn counters
  "Counters of every cluster of the handle, reduced over its devices (SUM; first violation MIN;
  payload maximum MAX)."
  [sim]
  (let [m (Memory. counters-size)]
    (call "raft_sim_read_counters" (:ptr sim) m)
    (merge (zipmap counter-names (for [i (range (count counter-names))] (.getLong m (+ 16 (* 8 i)))))
           {:node-ticks (.getLong m 0)
            :first-violation-tick (let [v (.getLong m 8)] (when-not (= v -1) v))
            :payload-max (.getLong m 240)})))

(defn digest
  "Per-cluster FNV-1a-64 of the canonical state (SIM_SPEC §6) for clusters [c0, c0+nc)."
  [sim c0 nc]
  (let [m (Memory. (* 8 nc))]
    (call "raft_sim_digest" (:ptr sim) (int c0) (int nc) m)
    (vec (for [i (range nc)] (.getLong m (* 8 i))))))

(defn destroy! [sim]
  (.invokeVoid (f "raft_sim_destroy") (object-array [(:ptr sim)])))
