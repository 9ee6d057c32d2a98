;; The Clojure side of the drop-in (SURVEY.md §8f F1): raft.sim over libraftsim.so through JNA, and
;; raft.sim.harness, which drives the reference's own raft.core/wait under seeded hooks. It sits
;; next to the reference's project (Clojure 1.6, core.async 0.1.278; project.clj:6-14 there) and
;; adds only JNA. Untested in this image (no JVM); tests/test_clojure_facade.py checks its struct
;; offsets and ABI symbol names against include/raftsim.h.
(defproject raft-sim-mi355x "0.2.0"
  :description "Batched MI355X Raft simulation behind raft.core's node loop"
  :dependencies [[org.clojure/clojure "1.6.0"]
                 [org.clojure/core.async "0.1.278.0-76b25b-alpha"]
                 [net.java.dev.jna/jna "5.13.0"]]
  :jvm-opts ["-Djna.library.path=../raft-simulation_amd/build"])
