(ns raft.sim.harness
  "Seeded hook harness: runs the reference's OWN handlers (raft.core/wait, core.clj:176-195) one
  event at a time under the discrete model of SIM_SPEC.md, so the literal reference's trace can be
  compared with raft.sim's (or the CPU oracle's) for the same seed and cluster id. Clojure 1.6 has
  no direct linking, so with-redefs reaches every call made inside wait:

    raft.server/incoming-rpc, raft.client/response-rpc -> chans holding at most the one message
                                  SIM_SPEC §4 P1 picked for this tick (the Philox EVENT bit decides
                                  between req and res, core.clj:181), so alts!! is deterministic
    raft.core/generate-timeout -> a closed chan when no message was picked (the D4 deadline is
                                  due: alts!! returns nil, the timeout branch), else a never-ready
                                  chan
    raft.client/rpc            -> capture [dst body] into the tick's outbox (client.clj:34)
    respond / redirect-client  -> land on the request's :resp-chan, read back after wait returns

  The caller feeds each tick's outbox through SIM_SPEC §4 P2 (delivery, faults) and draws the
  next deadline with `timeout-deadline`. Untested in this image: it has no JVM."
  (:require [clojure.core.async :as async]
            [raft.core :as core]
            [raft.client :as client]
            [raft.server :as server]))

(def ^:private M32 0xFFFFFFFF)

(defn philox
  "Philox4x32-10 (SIM_SPEC §5): counter [c0 c1 c2 c3], key [k0 k1] -> 4 words."
  [[c0 c1 c2 c3] [k0 k1]]
  (loop [r 0 c0 c0 c1 c1 c2 c2 c3 c3 k0 k0 k1 k1]
    (if (= r 10)
      [c0 c1 c2 c3]
      (let [p0 (* 0xD2511F53 c0) p1 (* 0xCD9E8D57 c2)]
        (recur (inc r)
               (bit-and (bit-xor (bit-shift-right p1 32) c1 k0) M32) (bit-and p1 M32)
               (bit-and (bit-xor (bit-shift-right p0 32) c3 k1) M32) (bit-and p0 M32)
               (bit-and (+ k0 0x9E3779B9) M32) (bit-and (+ k1 0xBB67AE85) M32))))))

(def ^:private EVENT 2)

(defn event-draw [{:keys [seed gid]} id t]
  (philox [gid (bit-or id (bit-shift-left EVENT 8)) t 0]
          [(bit-and seed M32) (bit-and (bit-shift-right seed 32) M32)]))

(defn timeout-deadline
  "generate-timeout (core.clj:171-174) as SIM_SPEC D4 draws it for the node map after the event."
  [{:keys [hb el-base el-span] :as sim} node t]
  (if (= (:state node) :leader)
    (+ t hb)
    (+ t el-base (bit-shift-right (* ((event-draw sim (:id node) t) 1) el-span) 32))))

(def ^:private request-types #{:request-vote :append-entries :client-set})

(defn- requester [message]
  (or (:candidate-id message) (:leader-id message)))

(defn wait-once
  "One `wait` of `node` with `message` (nil = the timeout branch). Returns [node' outbox], outbox
  holding [dst-id body] for every rpc and, for a request, [requester reply-or-redirect]."
  [system node message]
  (let [out (atom [])
        req (async/chan 1) res (async/chan 1) resp (async/chan 1)]
    (when message
      (if (request-types (:type message))
        (async/>!! req (assoc message :resp-chan resp))
        (async/>!! res message)))
    (with-redefs [server/incoming-rpc (constantly req)
                  client/response-rpc (constantly res)
                  core/generate-timeout (fn [_] (if message (async/chan) (doto (async/chan) async/close!)))
                  client/rpc (fn [_ cluster-node action body]
                               (swap! out conj [(:id cluster-node) (assoc body :type (keyword action))]))]
      (let [node' (core/wait system node)]
        (when (and message (request-types (:type message)))
          (let [[r port] (async/alts!! [resp] :default nil)]    ; a reply, unless none was sent
            (when (= port resp) (swap! out conj [(requester message) r]))))
        [node' @out]))))
