set -e
O=gpurun_out/settle; mkdir -p $O
timeout -k 10 120 python tools/settle_probe.py --steps 150 > $O/p0_first_process.json
timeout -k 10 120 python tools/settle_probe.py --churn-gib 200 > $O/c1.json
timeout -k 10 120 python tools/settle_probe.py --steps 150 > $O/p1_after_churn.json
timeout -k 10 120 python tools/settle_probe.py --steps 150 > $O/p2_next_process.json
timeout -k 10 120 python tools/settle_probe.py --churn-gib 200 > $O/c2.json
sleep 20
timeout -k 10 120 python tools/settle_probe.py --steps 150 > $O/p3_after_churn_sleep20.json
timeout -k 10 120 python tools/settle_probe.py --churn-gib 200 > $O/c3.json
timeout -k 10 120 python tools/settle_probe.py --steps 150 > $O/p4_after_churn.json
