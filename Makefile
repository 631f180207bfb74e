# The reference's src/model/KGAT/Makefile targets (train-sm, train, predict-sm, predict,
# recommend-sm) on the MI355X path; `make build` compiles libkgat_hip.so for gfx950.
PY ?= python
ARGS ?=

.PHONY: build train-sm train predict-sm predict recommend-sm recommend
build:
	$(PY) -c "import __graft_entry__ as g; g.build()"

train-sm:
	$(PY) tools/kgat_main.py --sm $(ARGS)

train:
	$(PY) tools/kgat_main.py $(ARGS)

predict-sm:
	$(PY) tools/kgat_main.py --sm --predict $(ARGS)

predict:
	$(PY) tools/kgat_main.py --predict $(ARGS)

recommend-sm:
	$(PY) tools/kgat_main.py --sm --recommend $(ARGS)

recommend:
	$(PY) tools/kgat_main.py --recommend $(ARGS)
