(ns raft.sim.harness
  "Seeded hook harness: runs the reference's OWN handlers (raft.core/wait, core.clj:176-195) under
  the discrete model of SIM_SPEC.md, so the literal reference's trace can be compared with the
  simulator's for the same seed and cluster id (SURVEY.md §8(b), F1). Clojure 1.6 has no direct
  linking, so with-redefs reaches every call made inside wait:

    raft.server/incoming-rpc, raft.client/response-rpc -> chans holding at most the one message
                                  SIM_SPEC §4 P1 picked for this tick (the Philox EVENT bit decides
                                  between req and res, core.clj:181), so alts!! is deterministic
    raft.core/generate-timeout -> a closed chan when no message was picked (the D4 deadline is
                                  due: alts!! returns nil, the timeout branch), else a never-ready
                                  chan
    raft.client/rpc            -> capture [dst body] into the tick's outbox (client.clj:34)
    clojure.core/rand-nth      -> the peer SIM_SPEC §4 draws from word 2 of the node's EVENT draw
                                  (client-set-handler's (rand-nth cluster), core.clj:154)
    respond / redirect-client  -> land on the request's :resp-chan, read back after wait returns
                                  (a ring response or a 302 whose Location names the target)

  `run-cluster` is the per-tick cluster driver of SIM_SPEC §4: P0 client injection (D9, D14), the
  D3 event choice and one wait per running node (P1), a Clojure exception inside wait halts the
  node with its pre-event state and no emission (D8: IndexOutOfBounds 1, NullPointer 2, ClassCast
  3, log capacity 4), D4 timer re-arm, then P2 delivery with the Philox fault draws (D5-D7, D12)
  and the client's redirect hops (D15). Payloads travel inside the messages as the reference's own
  entry vectors (no arena, so no eviction). `canonical-nodes` gives the canonical node tuples of
  raft.sim/nodes and tests/golden/*.json; `compare-golden` diffs a run against a golden fixture.
  All 32-bit word arithmetic is unchecked (unchecked-multiply, unsigned-bit-shift-right): checked
  long arithmetic overflows on Philox products. Untested in this image: it has no JVM."
  (:require [clojure.core.async :as async]
            [clojure.string :as str]
            [com.stuartsierra.component :as component]
            [raft.core :as core]
            [raft.client :as client]
            [raft.server :as server]
            [raft.log :as rlog]
            [clj-json.core :as json]))

(def ^:private M32 0xFFFFFFFF)
(def ^:private TWO32 4294967296)

(defn- mulhi
  "High word of the 64-bit product of two 32-bit words (the product is exact mod 2^64)."
  [a b]
  (unsigned-bit-shift-right (unchecked-multiply a b) 32))

(defn philox
  "Philox4x32-10 (SIM_SPEC §5): counter [c0 c1 c2 c3], key [k0 k1] -> 4 words."
  [[c0 c1 c2 c3] [k0 k1]]
  (loop [r 0 c0 c0 c1 c1 c2 c2 c3 c3 k0 k0 k1 k1]
    (if (= r 10)
      [c0 c1 c2 c3]
      (let [p0 (unchecked-multiply 0xD2511F53 c0) p1 (unchecked-multiply 0xCD9E8D57 c2)]
        (recur (inc r)
               (bit-and (bit-xor (unsigned-bit-shift-right p1 32) c1 k0) M32) (bit-and p1 M32)
               (bit-and (bit-xor (unsigned-bit-shift-right p0 32) c3 k1) M32) (bit-and p0 M32)
               (bit-and (unchecked-add k0 0x9E3779B9) M32)
               (bit-and (unchecked-add k1 0xBB67AE85) M32))))))

(def ^:private P-INIT 1)
(def ^:private P-EVENT 2)
(def ^:private P-NET 3)
(def ^:private P-CLIENT 4)
(def ^:private P-PART 6)

(defn- key-of [seed] [(bit-and seed M32) (bit-and (unsigned-bit-shift-right seed 32) M32)])

(defn- draw [{:keys [seed gid]} node purpose t extra]
  (philox [gid (bit-or node (bit-shift-left purpose 8)) t extra] (key-of seed)))

(defn event-draw [sim id t] (draw sim id P-EVENT t 0))

(defn- ppm [w] (mulhi w 1000000))

(defn timeout-deadline
  "generate-timeout (core.clj:171-174) as SIM_SPEC D4 draws it for the node map after the event."
  [{:keys [hb el-base el-span] :as sim} node t]
  (if (= (:state node) :leader)
    (unchecked-add t hb)
    (unchecked-add (unchecked-add t el-base) (mulhi ((event-draw sim (:id node) t) 1) el-span))))

;; ------------------------------------------------------------------ client model (SIM_SPEC P0)

(defn- client-powers
  "pw_i = (1-p)^(2^i) in 32-bit fixed point, truncating; client_ppm 0 keeps every power 2^32."
  [client-ppm]
  (let [pw0 (quot (unchecked-multiply (- 1000000 client-ppm) TWO32) 1000000)]
    (vec (take 32 (iterate (fn [p] (if (= p TWO32) p (mulhi p p))) pw0)))))

(defn- client-gap
  "G(w): the greedy search over the powers from 31 down to 0 (SIM_SPEC §4 P0)."
  [pw w]
  (let [u (inc w)]
    (loop [i 31 acc TWO32 g 0]
      (if (neg? i)
        g
        (let [p (pw i)
              c (cond (= acc TWO32) p
                      (= p TWO32) acc
                      :else (mulhi acc p))]
          (if (>= c u)
            (recur (dec i) c (unchecked-add g (bit-shift-left 1 i)))
            (recur (dec i) acc g)))))))

(defn- on-tick
  "tick(j) of the burst schedule, saturating at 2^32 - 1 (never)."
  [j period burst]
  (if (>= j M32)
    M32
    (let [t (if (pos? period) (unchecked-add (unchecked-multiply (quot j burst) period) (rem j burst)) j)]
      (min t M32))))

(defn- on-index [t period burst]
  (if (pos? period) (unchecked-add (unchecked-multiply (quot t period) burst) (rem t period)) t))

;; ------------------------------------------------------------------------ one wait of one node

(def ^:private request-types #{:request-vote :append-entries :client-set})

(defn- requester [message]
  (or (:candidate-id message) (:leader-id message)))

(defn- halt-code [^Throwable e]
  (cond (instance? IndexOutOfBoundsException e) 1
        (instance? NullPointerException e) 2
        (instance? ClassCastException e) 3
        :else (throw e)))

(defn- url->id [url] (- (Long/parseLong (last (str/split url #":"))) 8080))

(defn wait-once
  "One `wait` of `node` with `message` (nil = the timeout branch) and `w` the node's EVENT draw of
  this tick. Returns {:node node' :out [[dst body] ...] :reply [dst body] or nil :redirect id or
  nil :stdout text}, or {:halt code :stdout text} when the handler threw (D8)."
  [system node message w]
  (let [out (atom [])
        req (async/chan 1) res (async/chan 1) resp (async/chan 1)
        peers (:cluster system)]
    (when message
      (if (request-types (:type message))
        (async/>!! req (assoc message :resp-chan resp))
        (async/>!! res message)))
    (let [text (java.io.StringWriter.)
          result
          (binding [*out* text]
            (with-redefs [server/incoming-rpc (constantly req)
                          client/response-rpc (constantly res)
                          core/generate-timeout (fn [_] (if message
                                                          (async/chan)
                                                          (doto (async/chan) async/close!)))
                          client/rpc (fn [_ cluster-node action body]
                                       (swap! out conj [(:id cluster-node)
                                                        (assoc body :type (keyword action))]))
                          clojure.core/rand-nth (fn [coll]
                                                  (nth coll (mulhi (w 2) (count coll))))]
              (try
                {:node (core/wait system node)}
                (catch Exception e {:halt (halt-code e)}))))
          result (assoc result :stdout (str text))]
      (if (:halt result)
        result
        (let [r (when (and message (request-types (:type message)))
                  (first (async/alts!! [resp] :default nil)))]
          (cond-> (assoc result :out @out)
            (and r (= 302 (:status r))) (assoc :redirect (url->id (get-in r [:headers "Location"])))
            (and r (not= 302 (:status r))) (assoc :reply [(requester message) (:body r)])))))))

;; ----------------------------------------------------------------------------- cluster driver

(defn- msg-code [m]
  ({:request-vote 1 :append-entries 2 :client-set 3 :vote-response 4 :append-response 5}
   (:type m)))

(defn- msg-src [m] (or (:candidate-id m) (:leader-id m) (:id m) 0))

(defn- fnv [h w] (unchecked-multiply (bit-xor h w) 0x100000001B3))

(def ^:private FNV0 (.longValue 14695981039346656037N))

(def ^:private role-code {:follower 0 :candidate 1 :leader 2 :follwer 3})

(defn- trace-hash [h t ev src mterm node fault]
  (reduce fnv h [t ev src mterm (role-code (:state node)) (:current-term node) fault]))

(defn- insert
  "P2 insertion: stable by arrival, Q per queue counting messages in flight; halted receivers drop.
  A client-set's redirect hop count rides beside its body (not part of the printed message)."
  [st r which m arrival & [hops]]
  (let [q (get-in st [:queues r which])]
    (cond
      (pos? (get-in st [:fault r])) (update-in st [:counters :to-halted] inc)
      (>= (count q) (:inbox-cap st)) (update-in st [:counters :overflow] inc)
      :else (let [[a b] (split-with #(<= (:arrival %) arrival) q)]
              (-> st
                  (assoc-in [:queues r which] (vec (concat a [{:arrival arrival :msg m :hops (or hops 0)}] b)))
                  (update-in [:counters :delivered] inc))))))

(defn- queue-of [m] (if (request-types (:type m)) :req :res))

(defn- overflow?
  "The sim-only log capacity halt (SIM_SPEC §2): decided on the pre-event state, after every
  reference throw site of the handler."
  [st id node m]
  (let [L (:log-cap st)
        log (get-in st [:logs id])
        n (count (:entries @(:state log)))]
    (case (:type m)
      :append-entries (and (>= (:term m) (:current-term node))
                           (try (rlog/compare-prev? log (:prev-log-index m) (:prev-log-term m))
                                (catch Exception _ false))
                           (> (unchecked-add n (count (:entries m))) L))
      :client-set (and (= (:state node) :leader) (> (inc n) L))
      false)))

(defn- p1
  "One node's event at tick t: [st' emissions] with emissions [[dst body copies?] ...]."
  [st sim id t]
  (let [node (get-in st [:node id])
        {:keys [req res]} (get-in st [:queues id])
        req-ok (and (seq req) (<= (:arrival (first req)) t))
        res-ok (and (seq res) (<= (:arrival (first res)) t))
        w (event-draw sim id t)
        which (cond (and req-ok res-ok) (if (odd? (w 0)) :res :req)
                    req-ok :req res-ok :res
                    (>= t (get-in st [:deadline id])) :timeout
                    :else nil)]
    (if (nil? which)
      [st []]
      (let [head (when (not= which :timeout) (first (get-in st [:queues id which])))
            m (:msg head)
            st (if m (update-in st [:queues id which] (comp vec rest)) st)
            system {:client nil :server nil :log (get-in st [:logs id])
                    :cluster (for [p (range 1 (inc (:nodes st))) :when (not= p id)]
                               (core/cluster-node-info p))}
            seqno (get-in st [:seq id])
            ev (if m (msg-code m) (if (= (:state node) :leader) 7 6))
            src (if m (msg-src m) 0)
            mterm (if m (or (:term m) 0) 0)
            r (if (and m (overflow? st id node m))
                ;; the node map and message are printed before any handler runs (core.clj:182-186)
                {:halt 4
                 :stdout (with-out-str
                           (println "; Node") (prn node) (println "; Message")
                           (prn (if (request-types (:type m)) (assoc m :resp-chan (async/chan)) m))
                           (println ""))}
                (wait-once system node m w))
            ;; the printed channel identity is not reproducible: the node-local event number
            ;; stands in for it (SIM_SPEC §7)
            text (str/replace (:stdout r) #"ManyToManyChannel@[0-9a-f]+" (str "ManyToManyChannel@" (Long/toHexString seqno)))
            st (-> st (update-in [:stdout id] str text) (update-in [:seq id] inc))]
        (if-let [code (:halt r)]
          [(-> st
               (assoc-in [:fault id] code)
               (update-in [:trace id] trace-hash t ev src mterm node code))
           []]
          (let [node' (:node r)
                redirect (:redirect r)
                hops (:hops head 0)]
            [(-> st
                 (assoc-in [:node id] node')
                 (assoc-in [:deadline id] (timeout-deadline sim node' t))
                 (update-in [:trace id] trace-hash t ev src mterm node' 0))
             (concat (for [[dst body] (:out r)] [dst body :net])
                     (when-let [[dst body] (:reply r)] [[dst body :net]])
                     (when redirect
                       (if (< hops (:client-redirects st))
                         [[redirect {:command (:command m) :type :client-set} :client (inc hops)]]
                         [[nil nil :abandoned]])))]))))))

(defn- p2
  "Deliver the tick's emissions of sender s (in emission order) with the D5-D7/D12 fault draws."
  [st sim s t emissions]
  (let [{:keys [drop-ppm dup-ppm dmin dmax part-ppm part-epoch]} st
        part (draw sim 0 P-PART (quot t part-epoch) 0)
        parted (< (ppm (part 0)) part-ppm)
        span (unchecked-add (- dmax dmin) 1)]
    (reduce
      (fn [st [r body kind hops]]
        (case kind
          :abandoned (update-in st [:counters :client-abandoned] inc)
          :client (-> (update-in st [:counters :redirects] inc)
                      (insert r :req body (inc t) hops))
          :net
          (let [faulty (or (pos? drop-ppm) (pos? dup-ppm) (not= dmin dmax))
                w (if faulty (draw sim s P-NET t r) [0 0 0 0])
                st (update-in st [:counters :sent] inc)]
            (cond
              (and (pos? part-ppm) parted
                   (not= (bit-and (unsigned-bit-shift-right (part 1) s) 1)
                         (bit-and (unsigned-bit-shift-right (part 1) r) 1)))
              (update-in st [:counters :partitioned] inc)
              (and faulty (< (ppm (w 0)) drop-ppm)) (update-in st [:counters :dropped] inc)
              :else
              (let [d0 (unchecked-add dmin (mulhi (w 2) span))
                    st (insert st r (queue-of body) body (unchecked-add t d0))]
                (if (and faulty (< (ppm (w 1)) dup-ppm))
                  (-> (update-in st [:counters :duplicated] inc)
                      (insert r (queue-of body) body (unchecked-add t (unchecked-add dmin (mulhi (w 3) span)))))
                  st))))))
      st emissions)))

(defn- p0
  "Client injection (D9, D14): the cluster's next client-set, if it falls on tick t."
  [st sim t]
  (if (not= t (:client-next st))
    st
    (let [j (:client-count st)
          d (draw sim 0 P-CLIENT j 0)
          target (inc (mulhi (d 1) (:nodes st)))
          next-t (on-tick (unchecked-add (unchecked-add (on-index t (:client-period st) (:client-burst st)) 1)
                                         (client-gap (:pw st) (d 3)))
                          (:client-period st) (:client-burst st))]
      (-> st
          (update-in [:counters :client-injected] inc)
          (assoc :client-count (inc j) :client-next next-t)
          (insert target :req {:command (d 2) :type :client-set} t 0)))))

(def defaults
  {:nodes 5 :seed 42 :gid 0 :log-cap 64 :inbox-cap 16 :hb 3000 :el-base 5000 :el-span 5000
   :drop-ppm 0 :dup-ppm 0 :dmin 1 :dmax 1 :part-ppm 0 :part-epoch 1000 :client-ppm 0
   :client-period 0 :client-burst 1 :client-redirects 0})

(defn init-cluster
  "init-node (core.clj:31-38) and an empty Log (log.clj:33-34, writing to a temp file) for every
  node, D4 initial deadlines and the first client injection."
  [cfg]
  (let [st (merge defaults cfg)
        sim (select-keys st [:seed :gid :hb :el-base :el-span])
        ids (range 1 (inc (:nodes st)))
        pw (client-powers (:client-ppm st))
        first-c (if (pos? (:client-ppm st))
                  (on-tick (client-gap pw ((draw sim 0 P-CLIENT 0 1) 0))
                           (:client-period st) (:client-burst st))
                  M32)]
    (assoc st
      :sim sim :pw pw :client-next first-c :client-count 0
      :nodes-ids ids
      :node (into {} (for [i ids] [i (core/init-node i)]))
      :logs (into {} (for [i ids]
                       [i (component/start (rlog/create-log
                                             (str (java.io.File/createTempFile (str "node_" i) ".log"))))]))
      :deadline (into {} (for [i ids]
                           [i (unchecked-add (:el-base st)
                                             (mulhi ((draw sim i P-INIT 0 0) 1) (:el-span st)))]))
      :queues (into {} (for [i ids] [i {:req [] :res []}]))
      :fault (into {} (for [i ids] [i 0]))
      :trace (into {} (for [i ids] [i FNV0]))
      :seq (into {} (for [i ids] [i 0]))
      :stdout (into {} (for [i ids] [i ""]))
      :counters {:sent 0 :delivered 0 :dropped 0 :partitioned 0 :duplicated 0 :overflow 0
                 :to-halted 0 :client-injected 0 :redirects 0 :client-abandoned 0}
      :tick 0)))

(defn step-tick
  "SIM_SPEC §4 for one tick: P0, P1 for every running node (independently), P2."
  [st]
  (let [t (:tick st) sim (:sim st)
        st (p0 st sim t)
        [st ems] (reduce (fn [[st ems] id]
                           (if (pos? (get-in st [:fault id]))
                             [st ems]
                             (let [[st e] (p1 st sim id t)] [st (assoc ems id e)])))
                         [st {}] (:nodes-ids st))
        st (reduce (fn [st s] (p2 st sim s t (get ems s))) st (sort (keys ems)))]
    (assoc st :tick (inc t))))

(defn run-cluster
  "Run cluster `gid` of the configuration for `ticks` ticks from init-node."
  [cfg ticks]
  (nth (iterate step-tick (init-cluster cfg)) ticks))

(defn canonical-nodes
  "The canonical node tuples of raft.sim/nodes and tests/golden/*.json (SIM_SPEC §1, §6)."
  [st]
  (vec
    (for [id (:nodes-ids st)
          :let [n (get-in st [:node id])
                log @(:state (get-in st [:logs id]))
                entries (:entries log)
                ls (:leader-state n)
                peers (range 1 (inc (:nodes st)))
                mask (fn [s] (reduce bit-or 0 (map #(bit-shift-left 1 %) s)))
                keys* (filter #(and (contains? (:next-index ls) %) (contains? (:match-index ls) %))
                              peers)]]
      {:role (role-code (:state n))
       :voted_for (or (:voted-for n) 0)
       :leader_id (or (:leader-id n) 0)
       :fault (get-in st [:fault id])
       :entries_is_seq (if (vector? entries) 0 1)
       :ls_present (if ls 1 0)
       :votes (mask (:votes n))
       :ls_keys (mask keys*)
       :current_term (:current-term n)
       :commit_index (:commit-index log)
       :log_len (count entries)
       :deadline (get-in st [:deadline id])
       :next_index (vec (for [p peers] (if (some #{p} keys*) (get-in ls [:next-index p]) 0)))
       :match_index (vec (for [p peers] (if (some #{p} keys*) (get-in ls [:match-index p]) 0)))
       :trace_hash (format "%016x" (get-in st [:trace id]))
       :req_count (count (get-in st [:queues id :req]))
       :res_count (count (get-in st [:queues id :res]))
       :log (vec (for [e entries] [(:term e) (:val e)]))})))

(def ^:private golden-fields
  [:role :voted_for :leader_id :fault :entries_is_seq :ls_present :votes :ls_keys :current_term
   :commit_index :log_len :deadline :next_index :match_index :trace_hash :req_count :res_count :log])

(defn compare-golden
  "Run a tests/golden/*.json fixture's configuration through the reference's own handlers and
  return the differences from the fixture: final node fields, and the printed `; Node` /
  `; Message` trace of every node where the fixture holds one (BASELINE config 1: c1_seed42)."
  [path]
  (let [fx (json/parse-string (slurp path) true)
        cfg (reduce-kv (fn [m k v] (assoc m (keyword (str/replace (name k) "_" "-")) v))
                       {} (:config fx))
        st (run-cluster (assoc cfg :gid (:cluster_offset fx)) (:ticks fx))
        got (canonical-nodes st)]
    (concat
      (for [[i want] (map-indexed vector (:nodes fx))
            f golden-fields
            :let [g (get-in got [i f]) w (get want f)]
            :when (not= g w)]
        {:node (inc i) :field f :harness g :golden w})
      (for [[i text] (:stdout fx)
            :let [id (Long/parseLong (name i))]
            :when (not= text (get-in st [:stdout id]))]
        {:node id :field :stdout
         :first-difference (count (take-while true? (map = text (get-in st [:stdout id]))))}))))
