source tools/diag5.sh
run c3 c3 A=1 && run c3_notrace c3 NWK_NOTRACE=1 && run c4 c4 A=1 && run big13 big13 A=1 && run c3_o0 c3 NWK_ORDER=0
