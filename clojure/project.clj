;; The Clojure side of the drop-in (SURVEY.md §8f F1): raft.sim over libraftsim.so through JNA, and
;; raft.sim.harness, which drives the reference's own raft.core/wait under seeded hooks. It sits
;; next to the reference's project (Clojure 1.6, core.async 0.1.278; project.clj:6-14 there) and
;; adds only JNA. Untested in this image (no JVM); tests/test_clojure_facade.py checks its struct
;; offsets and ABI symbol names against include/raftsim.h, and the harness's arithmetic statically.
;;
;; The harness profile puts the reference's own sources (angelini/raft-simulation src/, path from
;; RAFT_REFERENCE_SRC) and its dependencies on the classpath:
;;   RAFT_REFERENCE_SRC=/path/to/raft-simulation/src lein with-profile +harness repl
;;   (require 'raft.sim.harness)
;;   (raft.sim.harness/compare-golden "../tests/golden/c1_seed42.json")   ; () = trace-equal
(defproject raft-sim-mi355x "0.3.0"
  :description "Batched MI355X Raft simulation behind raft.core's node loop"
  :dependencies [[org.clojure/clojure "1.6.0"]
                 [org.clojure/core.async "0.1.278.0-76b25b-alpha"]
                 [net.java.dev.jna/jna "5.13.0"]]
  :jvm-opts ["-Djna.library.path=../raft-simulation_amd/build"]
  :profiles {:harness
             {:source-paths [~(or (System/getenv "RAFT_REFERENCE_SRC") "../../raft-simulation/src")]
              :dependencies [[org.clojure/math.numeric-tower "0.0.4"]
                             [com.stuartsierra/component "0.2.1"]
                             [clj-http "0.9.1"]
                             [clj-json "0.5.3"]
                             [ring/ring-core "1.2.2"]
                             [ring/ring-json "0.3.0"]
                             [ring/ring-jetty-adapter "1.2.2"]]}})
