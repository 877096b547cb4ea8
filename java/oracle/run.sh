#!/usr/bin/env bash
# Runs LuceneGolden against real lucene-core where a JDK ≥ 22 exists; not in this image.
#   LUCENE_JAR=/path/lucene-core-10.3.0.jar bash java/oracle/run.sh /tmp/lg
# (the jar is the version the reference pins: gradle/libs.versions.toml:3)
set -euo pipefail
dir=${1:?case directory written by golden_io.py export}
jar=${LUCENE_JAR:?set LUCENE_JAR to lucene-core-10.3.0.jar}
here=$(cd "$(dirname "$0")" && pwd)
out=$(mktemp -d)
javac -cp "$jar" -d "$out" "$here/LuceneGolden.java"
# Panama VectorUtil (the order the CPU baseline restates) needs the incubator module
java --add-modules jdk.incubator.vector -cp "$jar:$out" LuceneGolden "$dir"
